#!/bin/bash
# round 4, final kernel: configs[3]'s flow at 65,536 / 131,072 / 262,144 envs per GPU, then
# configs[0]'s exact shape (one Environment, 1,000 warm-up + 10,000 timed step(0))
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04ah
mkdir -p $O
for n in 65536 131072 262144; do
  timeout -k 10 300 python bench.py --workload config4 --envs $n --steps 20 --warmup 2 --no-cpu-baseline > $O/config4_$n.json 2>> $O/err.log || exit 1
done
timeout -k 10 800 python -u bench.py --workload config1 > $O/config1_full.json 2> $O/config1_full.err
echo "exit=$?" > $O/exit.txt
