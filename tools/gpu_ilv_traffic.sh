#!/bin/bash
# HBM-side traffic (FETCH_SIZE / WRITE_SIZE passes) of K1 at the image interleave chosen per handle
# (= K1's envs per wave) and at the 64-env interleave of rounds 1-2 (PK_ILV=64), for config3 and
# config4 (one sub-batch, so each dispatch is the whole shard); plus the calibration copies.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ilvtraffic_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/cfetch -o cfetch --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cfetch.out 2> $OUT/cfetch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/cwrite -o cwrite --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cwrite.out 2> $OUT/cwrite.err || { echo "exit=calib" > $OUT/exit.txt; exit 1; }
rc=0
for w in "config3|--workload config3" "config4|--workload config4 --batches 1"; do
  name=${w%%|*}; args=${w#*|}
  for ilv in auto 64; do
    D=$OUT/${name}_$ilv; mkdir -p $D
    if [ $ilv = 64 ]; then export PK_ILV=64; else unset PK_ILV; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o fetch --output-format csv -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/fetch_bench.json 2> $D/fetch.err && \
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/write -o write --output-format csv -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $args > $D/write_bench.json 2> $D/write.err || { rc=$?; break 2; }
  done
done
unset PK_ILV
echo "exit=$rc" > $OUT/exit.txt
