#!/bin/bash
# round 4 final kernel, part 2: the horizon test file, then the round profile (rocprofv3 stats +
# PMC passes of every workload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04ag2
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_horizon.py -m gpu --durations=10 > gpurun_out/r04ag2/pytest_horizon.log 2>&1 || { echo "exit=$?" > gpurun_out/r04ag2/exit.txt; exit 1; }
bash tools/gpu_round_prof.sh r04ag "config2|--workload config2" "config3|--workload config3" "config4|--workload config4" "config5|--workload config5"
echo "exit=$?" > gpurun_out/r04ag2/exit.txt
