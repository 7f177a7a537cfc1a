#!/bin/bash
# Round-final bench lines: the driver's default command (config3 with the CPU baseline), every
# workload without it, the 64-bank ROM, and throughput vs envs per GPU (configs[3] shard sizes of
# N = 8, 4, 2, 1).  Each GPU step has its own time limit; the chain stops at the first failure.
# usage: bash tools/gpu_round_bench.sh TAG   (outputs in gpurun_out/rbench_TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rbench_${1:-x}
mkdir -p $OUT
cd $R
B="timeout -k 10 400 python bench.py"
$B > $OUT/default.json 2> $OUT/err.log && \
$B --no-cpu-baseline --workload config2 > $OUT/config2.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config4 > $OUT/config4.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config5 > $OUT/config5.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config3 --rom-banks 64 > $OUT/config3_b64.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config4 --rom-banks 64 > $OUT/config4_b64.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config4 --envs 65536 --steps 10 > $OUT/config4_n65536.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config4 --envs 131072 --steps 8 > $OUT/config4_n131072.json 2>> $OUT/err.log && \
$B --no-cpu-baseline --workload config4 --envs 262144 --steps 4 --warmup 1 > $OUT/config4_n262144.json 2>> $OUT/err.log
rc=$?
echo "exit=$rc" > $OUT/exit.txt
exit $rc
