#!/bin/bash
# round 4, third GPU call: the 78 KB-LDS K1 (two workgroups per CU) with more VecEnv sub-batches
# (hardware queues raised so every sub-batch stream has its own), and on configs[2]/[4]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIBS="cur lds2" WLS="config3 config5" STEPS=8 tools/gpu_ab.sh r04c_c35 || exit 1
LIBS="cur@GPU_MAX_HW_QUEUES=8 lds2@GPU_MAX_HW_QUEUES=8" WLS="config4" STEPS=8 BENCH_EXTRA="--batches 4" tools/gpu_ab.sh r04c_b4 || exit 1
LIBS="lds2@GPU_MAX_HW_QUEUES=12" WLS="config4" STEPS=8 BENCH_EXTRA="--batches 8" tools/gpu_ab.sh r04c_b8 || exit 1
LIBS="cur lds2 lds2@GPU_MAX_HW_QUEUES=8" WLS="config4" STEPS=8 BENCH_EXTRA="--batches 2" tools/gpu_ab.sh r04c_b2 || exit 1
