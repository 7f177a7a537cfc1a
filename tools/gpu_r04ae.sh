#!/bin/bash
# the frame watchdog folded into the tick limit (386 -> 381 issued) + the watchdog parity test: parity + A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04ae
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_wd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04ae/parity.log 2>&1 || exit $?
LIBS="base wd" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04ae || exit $?
LIBS="base wd" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04ae_c2 || exit $?
