#!/bin/bash
# Quick GPU iteration: parity tests + bench workloads (no profiler).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu-baseline $BENCH_EXTRA > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 python bench.py --workload config5 --steps 10 --no-cpu-baseline > $OUT/bench_config5.json 2>> $OUT/bench.err && \
timeout -k 10 600 python bench.py --workload config2 --envs 4096 --no-cpu-baseline > $OUT/bench_config2.json 2>> $OUT/bench.err
echo "exit=$?" > $OUT/check.log
