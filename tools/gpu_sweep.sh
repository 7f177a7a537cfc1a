#!/bin/bash
# K1 wave-shape sweep: PK_WAVE_LANES per workload (bench, no profiler).  usage: bash tools/gpu_sweep.sh TAG "wl:lanes ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
OUT=$R/gpurun_out/sweep_$TAG
mkdir -p $OUT
cd $R
rc=0
for item in $2; do
  w=${item%%:*}; l=${item##*:}
  PK_WAVE_LANES=$l timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --workload $w $SWEEP_EXTRA > $OUT/${w}_l$l.json 2>> $OUT/err.log || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
