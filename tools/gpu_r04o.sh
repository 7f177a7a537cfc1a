#!/bin/bash
# round 4: configs[0]'s exact shape (test.py:16-29): one Environment, 1,000 warm-up + 10,000 timed step(0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04o
timeout -k 10 1000 python -u bench.py --workload config1 > gpurun_out/r04o/config1_full.json 2> gpurun_out/r04o/config1_full.err
echo "exit=$?" > gpurun_out/r04o/exit.txt
