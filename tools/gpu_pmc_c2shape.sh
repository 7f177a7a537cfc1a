#!/bin/bash
# configs[1] (config2: 4,096 lockstep envs, headless) in its default shape (32 envs per wave, 128
# waves on 32 CUs) and spread over every CU (4 envs per wave, 1,024 waves): the same counter passes
# for both, to name what makes the spread shape 2.7x slower per wave iteration.
# usage: bash tools/gpu_pmc_c2shape.sh TAG   (outputs in gpurun_out/pmcc2_TAG/{default,spread}_pN)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcc2_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # shape pass counters...
  local shape=$1 p=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/${shape}_$p -o $p --output-format csv -- \
      python3 $R/bench.py --workload config2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${shape}_$p.json 2> $OUT/${shape}_$p.err
}
passes() {
  local shape=$1
  run $shape p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES && \
  run $shape p2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS && \
  run $shape p3 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum && \
  run $shape p4 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum && \
  run $shape p5 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
}
passes default && \
( export PK_WAVE_LANES=4 PK_K1_BLOCK=256; passes spread )
echo "exit=$?" > $OUT/exit.txt
