#!/bin/bash
# Run-to-run spread of the headline line: the driver's default `python bench.py` (configs[3],
# CPU baseline included) five times back to back on one box, then configs[2] three times without
# the CPU leg.  Each GPU step has its own time limit; the chain stops at the first failure.
# usage: bash tools/gpu_repeat_bench.sh TAG   (outputs in gpurun_out/repeat_TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/repeat_${1:-x}
mkdir -p $OUT
cd $R
B="timeout -k 10 400 python bench.py"
$B > $OUT/default_1.json 2> $OUT/err.log && \
$B > $OUT/default_2.json 2>> $OUT/err.log && \
$B > $OUT/default_3.json 2>> $OUT/err.log && \
$B > $OUT/default_4.json 2>> $OUT/err.log && \
$B > $OUT/default_5.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config2 > $OUT/config2_1.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config2 > $OUT/config2_2.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config2 > $OUT/config2_3.json 2>> $OUT/err.log
rc=$?
echo "exit=$rc" > $OUT/exit.txt
exit $rc
