#!/bin/bash
# Bench every workload once (no profiler) after an optional test pass; each GPU step has its own
# time limit and the chain stops at the first failure.  usage: bash tools/gpu_bench_all.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
OUT=$R/gpurun_out/bench_$TAG
mkdir -p $OUT
cd $R
B="timeout -k 10 400 python bench.py --no-cpu-baseline"
( [ -z "$PYTEST_K" ] || timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1 ) && \
$B --workload config3 > $OUT/config3.json 2> $OUT/err.log && \
$B --workload config2 > $OUT/config2.json 2>> $OUT/err.log && \
$B --workload config4 > $OUT/config4.json 2>> $OUT/err.log && \
$B --workload config5 > $OUT/config5.json 2>> $OUT/err.log && \
$B --workload config3 --rom-banks 64 > $OUT/config3_b64.json 2>> $OUT/err.log && \
$B --workload config4 --rom-banks 64 > $OUT/config4_b64.json 2>> $OUT/err.log
echo "exit=$?" > $OUT/exit.txt
