#!/bin/bash
# Instruction-mix / stall PMC passes of K1 (one rocprofv3 run per counter group, <=8 SQ counters each).
# usage: bash tools/gpu_pmc_mix.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH_ARGS="$*"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o $name --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/$name.json 2> $OUT/$name.err
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && \
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH && \
run c SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT
echo "exit=$?" >> $OUT/done.txt
