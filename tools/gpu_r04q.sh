#!/bin/bash
# ALL-banks-staged K1 instance: parity (hostsim-equal kernels on the GPU) + A/B against HEAD's K1
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04q
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_all.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04q/parity.log 2>&1 || exit $?
LIBS="base all" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04q_c2 || exit $?
LIBS="base all" WLS="config2 config4" STEPS=4 BENCH_EXTRA="--envs 131072" bash tools/gpu_ab.sh r04q_131k || exit $?
