#!/bin/bash
# Sanity (smoke + default bench) and a config2 K1 workgroup-size sweep (PK_K1_BLOCK / PK_WAVE_LANES).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/blk
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "exit=smoke $?" > $O/exit.txt; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "exit=bench $?" > $O/exit.txt; exit 1; }
for cfg in "0 0" "64 0" "128 0" "64 64" "128 64"; do
  set -- $cfg
  tag=b$1_l$2
  E=""
  [ "$1" != 0 ] && E="$E PK_K1_BLOCK=$1"
  [ "$2" != 0 ] && E="$E PK_WAVE_LANES=$2"
  env $E timeout -k 10 300 python bench.py --workload config2 --envs 4096 --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_$tag.json 2>> $O/err.log || { echo "exit=$tag $?" > $O/exit.txt; exit 1; }
done
echo "exit=0" > $O/exit.txt
