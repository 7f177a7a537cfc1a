#!/bin/bash
# loop-top rare stages behind one branch + unconditional second RAM byte load: parity + A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04s
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_top.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04s/parity.log 2>&1 || exit $?
LIBS="base top" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04s || exit $?
LIBS="base top" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04s_c2 || exit $?
