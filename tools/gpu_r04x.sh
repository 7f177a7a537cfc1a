#!/bin/bash
# wave-priority variant in the small-LDS K1 (VecEnv sub-batches, 2 waves per SIMD): A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
LIBS="cur cur@PK_K1_PRIO=1" WLS="config3 config4 config5" STEPS=6 bash tools/gpu_ab.sh r04x || exit $?
