#!/bin/bash
# register-file pin (no sinking past the prefetch), VM drains at rare-block ends (no vmcnt(0) at the
# loop top), branch-free buffer stores in the unstaged-bank instance (vmcnt(2) at the prefetch
# instead of waiting for the iteration's stores): parity of the last + A/B against HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r04w
PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_bst.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04w/parity.log 2>&1 || exit $?
LIBS="base pin drain bst" WLS="config3 config4" STEPS=6 bash tools/gpu_ab.sh r04w || exit $?
LIBS="base pin drain bst" WLS="config2" STEPS=8 bash tools/gpu_ab.sh r04w_c2 || exit $?
