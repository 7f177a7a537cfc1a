#!/bin/bash
# round 4: operand-independent control values and the fused-pair decision computed between the
# operand loads' issue and their wait (hoist) vs the previous library (dual); parity subset first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04n
PK_LIB=$R/pokegym_amd/lib/libpokegym_amd_hoist2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py::test_config4_flow_vs_oracle_per_env tests/test_gpu_scale.py::test_small_lds_kernel_48_steps -m gpu > gpurun_out/r04n/pytest.log 2>&1 || exit 1
LIBS="dual hoist hoist2" WLS="config3 config4 config2" STEPS=10 tools/gpu_ab.sh r04n || exit 1
