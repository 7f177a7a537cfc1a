#!/bin/bash
# round 4: the configs[4] VecEnv flow vs the oracle per env, then the multi-rank bench rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_scale.py::test_config5_flow_vecenv_vs_oracle_per_env > gpurun_out/r04j/pytest.log 2>&1 || exit 1
bash tools/gpu_rehearse_multi.sh
