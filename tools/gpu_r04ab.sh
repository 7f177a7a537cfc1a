#!/bin/bash
# fuse length check as one compare against the bytes available (403 -> 396 issued): parity + A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04ab
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_len.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04ab/parity.log 2>&1 || exit $?
LIBS="base len" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04ab || exit $?
LIBS="base len" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04ab_c2 || exit $?
