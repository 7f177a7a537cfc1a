#!/bin/bash
# round 4 final kernel: the 1 MiB (64-bank) pkbench layout on configs[2] and configs[3]'s shard
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04ai
mkdir -p $O
for w in config3 config4; do
  timeout -k 10 300 python bench.py --workload $w --rom-banks 64 --steps 20 --warmup 2 --no-cpu-baseline > $O/${w}_64banks.json 2>> $O/err.log || exit 1
done
echo "exit=0" > $O/exit.txt
