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
  run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT && \
  run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
