#!/bin/bash
# LDS bank-conflict counters of K1 (microcode entries are 64 B apart: a ds_read_b128 lane group of
# 16 divergent lanes maps onto 4 of the 16 slots of a 256-B bank row)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmclds_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name workload counters...
  local name=$1 w=$2; shift 2
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o $name --output-format csv -- \
      python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err
}
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
run c2 config2 $C && run c3 config3 $C && run c4 config4 $C
echo "exit=$?" > $OUT/exit.txt
