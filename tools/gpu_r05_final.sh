#!/bin/bash
# Round-5 final kernel evidence in two GPU sessions (each fits one gpurun call):
#   prof  rocprofv3 kernel-trace stats of the driver's exact default command, then the round profile
#         of every workload (stats + PMC passes, tools/gpu_round_prof.sh)
#   prof2 the same profile of config2 and the 64-bank config3
#   bench the bench lines (tools/gpu_round_bench.sh) and configs[0]'s shape (config1, 1,000 +
#         10,000 x step(0))
# Each GPU step has its own time limit; the chain stops at the first failure.
# usage: bash tools/gpu_r05_final.sh prof|prof2|bench TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${2:-r05f}
OUT=$R/gpurun_out/drv_$TAG
mkdir -p $OUT
if [ "$1" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o stats --output-format csv -- \
      python3 $R/bench.py > $OUT/driver_cmd_bench_under_rocprof.json 2> $OUT/driver_cmd.err && \
  bash $R/tools/gpu_round_prof.sh $TAG "config3|--workload config3" "config4|--workload config4" \
      "config5|--workload config5"
elif [ "$1" = prof2 ]; then
  bash $R/tools/gpu_round_prof.sh ${TAG}b "config2|--workload config2" "config3_b64|--workload config3 --rom-banks 64"
else
  bash $R/tools/gpu_round_bench.sh $TAG && \
  cd $R && timeout -k 10 900 python bench.py --workload config1 > $OUT/config1_full.json 2> $OUT/config1.err
fi
rc=$?
echo "exit=$rc" > $OUT/exit_$1.txt
exit $rc
