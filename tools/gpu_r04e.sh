#!/bin/bash
# round 4: bench lines of every workload with config3/config5 stepped through VecEnv (2 sub-batches),
# the bench contract test, and the configs[1] shape PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04e
mkdir -p $O
LIBS="dual" WLS="config3 config4 config5 config2" STEPS=20 tools/gpu_ab.sh r04e_bench || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bench_contract.py -m gpu > $O/contract.log 2>&1 || exit 1
bash tools/gpu_pmc_c2shape.sh r04e
