#!/bin/bash
# GPU parity session: smoke, then the -m gpu tests of $TESTS (default: all of tests/) with a per-test
# timeout (thread method, so a hang names its test).  The whole suite takes longer than one gpurun
# call: split it, e.g. TESTS=tests/test_gpu_horizon.py and PYTEST_EXTRA="--ignore=tests/test_gpu_horizon.py".
# usage: bash tools/gpu_tests.sh TAG  (outputs in gpurun_out/tests_TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tests_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 ${PYTEST_LIMIT:-1050} python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread $PYTEST_EXTRA > $OUT/pytest_gpu.log 2>&1
echo "exit=$?" > $OUT/exit.txt
