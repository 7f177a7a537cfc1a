#!/bin/bash
# Round checkpoint: smoke, the whole -m gpu suite, then every bench line (default = with the CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > $OUT/bench_config4.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > $OUT/bench_config2.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config3 --rom-banks 64 --no-cpu-baseline > $OUT/bench_config3_b64.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config4 --rom-banks 64 --no-cpu-baseline > $OUT/bench_config4_b64.json 2>> $OUT/bench.err
echo "exit=$?" > $OUT/exit.txt
