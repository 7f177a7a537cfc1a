#!/bin/bash
# Final bench lines of every workload (default = with the CPU baseline), then round profiles of the
# 32,768-env shard workloads (16-env waves, two per SIMD, since this kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/final_r02q
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > $OUT/bench_config4.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > $OUT/bench_config2.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config3 --rom-banks 64 --no-cpu-baseline > $OUT/bench_config3_b64.json 2>> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config4 --rom-banks 64 --no-cpu-baseline > $OUT/bench_config4_b64.json 2>> $OUT/bench.err || { echo "exit=bench $?" > $OUT/exit.txt; exit 1; }
echo "exit=0" > $OUT/exit.txt
bash tools/gpu_round_prof.sh r02q "config4|--workload config4" "config5|--workload config5"
