#!/bin/bash
# VecEnv sub-batch count with the small-LDS K1: 2 (default) vs 4 vs 8 (GPU_MAX_HW_QUEUES=12 so every
# sub-batch stream has its own hardware queue), ABAB
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/ab_r04aa
mkdir -p $O
for rep in 1 2; do
  for w in config3 config4; do
    for b in 2 4 8; do
      GPU_MAX_HW_QUEUES=12 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --workload $w --batches $b > $O/${w}_b${b}_$rep.json 2>> $O/err.log || exit 1
    done
  done
done
