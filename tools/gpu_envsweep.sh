#!/bin/bash
# Throughput vs envs per GPU (config3 shape, default wave shape per size).  usage: bash tools/gpu_envsweep.sh TAG "32768 65536 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
OUT=$R/gpurun_out/envsweep_$TAG
mkdir -p $OUT
cd $R
rc=0
for n in $2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-6} --warmup 2 --workload ${WL:-config3} --envs $n $SWEEP_EXTRA > $OUT/${WL:-config3}_n$n.json 2>> $OUT/err.log || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
