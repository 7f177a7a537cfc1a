#!/bin/bash
# rlim (one-compare staged-ROM test), the staged-bank order (blank banks last) and the hoisted
# tick bookkeeping: parity of the last + A/B against HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04r
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_tick.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04r/parity.log 2>&1 || exit $?
LIBS="base rlim order order@PK_STAGE_BANKS=3 tick" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04r || exit $?
LIBS="base rlim tick" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04r_c2 || exit $?
