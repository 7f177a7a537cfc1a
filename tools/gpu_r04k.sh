#!/bin/bash
# round 4: memory-free DIV/JOYP IO reads (io1) vs the previous library (dual); parity subset first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py::test_config4_flow_vs_oracle_per_env -m gpu > gpurun_out/r04k/pytest.log 2>&1 || exit 1
LIBS="dual io1" WLS="config3 config4 config2" STEPS=10 tools/gpu_ab.sh r04k || exit 1
