#!/bin/bash
# Round-final kernel evidence in GPU sessions that each fit one gpurun call:
#   prof  rocprofv3 kernel-trace stats of the driver's exact default command, then the round profile
#         of every workload (stats + PMC passes, tools/gpu_round_prof.sh)
#   prof2 the same profile of config2 and the 64-bank config3
#   bench the bench lines (tools/gpu_round_bench.sh) and configs[0]'s shape (config1, 1,000 +
#         10,000 x step(0))
#   conc  the PMC record of configs[2] at the occupancy its timed steps run (two small-LDS K1
#         workgroups per CU = two 32-env waves per SIMD) as ONE launch: the whole 65,536-env handle
#         through the small-LDS kernel (PK_K1_SMALL=1, VecEnv with one batch) — rocprofv3 --pmc
#         serialises dispatches, so the bench's two concurrent sub-batch launches are profiled one
#         at a time (one wave per SIMD) in the prof session; likewise configs[3]/[4]'s shards
#         (config4/config5: 32,768 envs in 16-env waves, two per SIMD)
#   stamp phase stamps (-DPK_STAMP build, whole-handle launches; config3small = the small-LDS
#         kernel the VecEnv sub-batches run, at their two-waves-per-SIMD occupancy)
# Each GPU step has its own time limit; the chain stops at the first failure.
# usage: bash tools/gpu_round_final.sh prof|prof2|bench|conc|stamp TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${2:-r06}
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
elif [ "$1" = conc ]; then
  PK_K1_SMALL=1 bash $R/tools/gpu_round_prof.sh ${TAG}c "config3_2wps|--workload config3 --batches 1" \
      "config4_2wps|--workload config4 --batches 1" "config5_2wps|--workload config5 --batches 1"
elif [ "$1" = stamp ]; then
  cd $R && bash tools/gpu_stamp.sh $TAG "config3small|PK_K1_SMALL=1 --workload config3" "config3|--workload config3" \
      "config4|--workload config4" "config2|--workload config2"
else
  bash $R/tools/gpu_round_bench.sh $TAG && \
  cd $R && timeout -k 10 900 python bench.py --workload config1 > $OUT/config1_full.json 2> $OUT/config1.err
fi
rc=$?
echo "exit=$rc" > $OUT/exit_$1.txt
exit $rc
