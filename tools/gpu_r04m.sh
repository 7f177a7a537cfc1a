#!/bin/bash
# round 4: the 10k-step horizon file incl. the small-LDS kernel shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04m
timeout -k 10 1120 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_horizon.py -m gpu --durations=10 > gpurun_out/r04m/pytest_horizon.log 2>&1
echo "exit=$?" > gpurun_out/r04m/exit.txt
