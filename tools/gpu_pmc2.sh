#!/bin/bash
# memory-pipeline counters (TA/TCP/UTCL1); usage: bash tools/gpu_pmc2.sh TAG [bench args]
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
run m1 TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_SERIALIZATION_STALL && \
run m2 TCP_TOTAL_CACHE_ACCESSES TCP_CACHE_MISS TCP_PENDING_STALL_CYCLES TCP_TCP_TA_ADDR_STALL_CYCLES && \
run m3 TA_TA_BUSY TA_TOTAL_WAVEFRONTS TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES && \
run m4 TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TOTAL_READ
echo "exit=$?" >> $OUT/done.txt
