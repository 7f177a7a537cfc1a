#!/bin/bash
# unmasked DIV accumulator sums, unconditional instruction count (381 -> 379 issued) + instruction-count parity tests: parity + A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04af
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_ic.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04af/parity.log 2>&1 || exit $?
LIBS="base ic" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04af || exit $?
LIBS="base ic" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04af_c2 || exit $?
