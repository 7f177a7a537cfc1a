#!/bin/bash
# Round-final profile of every workload: rocprofv3 kernel-trace stats of the bench, then separate PMC
# passes (FETCH_SIZE; WRITE_SIZE; VALU/stall counters) and, once, the 1 GiB copy that calibrates the
# FETCH/WRITE units (MI355X_MICROARCH.md §HBM).  usage: bash tools/gpu_round_prof.sh TAG "wname|bench args" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/rprof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rc=0
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/cfetch -o cfetch --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cfetch.out 2> $OUT/cfetch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/cwrite -o cwrite --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cwrite.out 2> $OUT/cwrite.err || { echo "exit=calib" > $OUT/exit.txt; exit 1; }
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  D=$OUT/$name
  mkdir -p $D
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/stats -o stats --output-format csv -- \
      python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > $D/stats_bench.json 2> $D/stats.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o fetch --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/fetch_bench.json 2> $D/fetch.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/write -o write --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/write_bench.json 2> $D/write.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $D/valu -o valu --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/valu_bench.json 2> $D/valu.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM -d $D/issue -o issue --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/issue_bench.json 2> $D/issue.err || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
exit $rc
