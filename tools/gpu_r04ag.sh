#!/bin/bash
# round-4 validation of the final kernel, part 1: smoke + every -m gpu test but the horizon file,
# bench lines of configs[1..4], then the driver's exact default bench command under rocprofv3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04ag
mkdir -p $O
TESTS=tests PYTEST_EXTRA="--ignore=tests/test_gpu_horizon.py" PYTEST_LIMIT=600 bash tools/gpu_tests.sh r04ag
grep -q "exit=0" gpurun_out/tests_r04ag/exit.txt || exit 1
REPS=1 LIBS="fin" WLS="config3 config4 config5 config2" STEPS=20 bash tools/gpu_ab.sh r04ag_bench || exit 1
bash tools/gpu_final_stats.sh r04ag
