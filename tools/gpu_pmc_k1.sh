#!/bin/bash
# K1 issue/stall/clock PMC passes (one rocprofv3 run per counter group) for several bench
# variants.  usage: bash tools/gpu_pmc_k1.sh TAG "name|ENV=.. bench args" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmck_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -f $OUT/counters.txt ] || timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
rc=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}
  envs=""; args=""
  for tok in $rest; do case $tok in *=*) envs="$envs $tok";; *) args="$args $tok";; esac; done
  run() {
    local p=$1; shift
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/${name}_$p -o $p --output-format csv -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $OUT/${name}_$p.json 2> $OUT/${name}_$p.err
  }
  if [ -n "$MEMPASS" ]; then
    run c TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum && \
    run d TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum || { rc=$?; break; }
    continue
  fi
  if [ -n "$TAPASS" ]; then
    run g TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT && \
    run h TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_SPI_STALL_sum TD_LOAD_WAVEFRONT_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE || { rc=$?; break; }
    continue
  fi
  if [ -n "$ISSUEPASS" ]; then
    run e SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR && \
    run f SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY || { rc=$?; break; }
    continue
  fi
  run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT && \
  run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
