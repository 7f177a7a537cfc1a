#!/bin/bash
# K1 launch-shape sweep of one workload on the committed kernel: each spec is "tag|ENV=.. ENV=..".
# usage: WL=config3 bash tools/gpu_shape_sweep.sh TAG "l64|PK_WAVE_LANES=64" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/shape_${1:-x}; shift; mkdir -p $O
rc=0
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --workload ${WL:-config3} $BENCH_EXTRA > $O/${name}_$rep.json 2>> $O/err.log || { rc=$?; break 2; }
  done
done
echo "exit=$rc" > $O/exit.txt
