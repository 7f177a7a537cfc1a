#!/bin/bash
# Instruction-fetch counters of K1 (after config2's spread shape showed 100x the instruction waits
# per wave): the counter list of this GPU, then one pass per workload/shape.
# usage: bash tools/gpu_pmc_ifetch.sh TAG   (outputs in gpurun_out/pmcif_TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcif_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run() {  # name workload counters...
  local name=$1 w=$2; shift 2
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o $name --output-format csv -- \
      python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err
}
C="SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU"
run c2_default config2 $C && \
( export PK_WAVE_LANES=4 PK_K1_BLOCK=256; run c2_spread config2 $C ) && \
run c3 config3 $C && \
run c4 config4 $C && \
run c2_icache config2 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ && \
( export PK_WAVE_LANES=4 PK_K1_BLOCK=256; run c2s_icache config2 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ ) && \
run c3_icache config3 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
echo "exit=$?" > $OUT/exit.txt
