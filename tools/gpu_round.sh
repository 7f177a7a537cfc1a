#!/bin/bash
# One GPU session: smoke, GPU tests, bench, rocprofv3 kernel stats. Every GPU step has its own
# time limit and the steps are chained with && so the first failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 python bench.py --workload config2 --envs 4096 --no-cpu-baseline > $OUT/bench_config2.json 2>> $OUT/bench.err && \
timeout -k 10 600 python bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.json 2>> $OUT/bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err)
echo "exit=$?" >> $OUT/session.log
