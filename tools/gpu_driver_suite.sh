#!/bin/bash
# Rehearsal of the driver's round-end GPU tiers on one box: exactly `python -m pytest tests/ -x -q
# -m gpu` (plus --durations=0, output only) and then __graft_entry__.smoke(), each timed.
# usage: bash tools/gpu_driver_suite.sh TAG   (outputs in gpurun_out/TAG: pytest.log, smoke.log, wall.txt)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-driver}
mkdir -p $OUT
cd $R
SECONDS=0
timeout -k 10 ${PYTEST_LIMIT:-1000} python -u -m pytest tests/ -x -q -m gpu --durations=0 > $OUT/pytest.log 2>&1
rc=$?
t1=$SECONDS
echo "pytest rc=$rc wall_s=$t1" > $OUT/wall.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc wall_s=$((SECONDS - t1))" >> $OUT/wall.txt
exit $rc
