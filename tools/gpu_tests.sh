#!/bin/bash
# GPU parity session: smoke, then every -m gpu test (per-test timeout, thread method so a hang names its test).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $PYTEST_EXTRA > $OUT/pytest_gpu.log 2>&1
echo "exit=$?" >> $OUT/tests_exit.log
