#!/bin/bash
# the tick limit (next LCD event / LCD-off frame end, 0 with the timer on) kept as a lane register (396 -> 386 issued): parity + A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04ac
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_lim.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04ac/parity.log 2>&1 || exit $?
LIBS="base lim" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04ac || exit $?
LIBS="base lim" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04ac_c2 || exit $?
