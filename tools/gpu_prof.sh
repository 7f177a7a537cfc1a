#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the default bench, then separate PMC passes
# (FETCH_SIZE; WRITE_SIZE) over the bench and over a 1 GiB copy used to calibrate the units.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o stats --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $OUT/stats_bench.json 2> $OUT/stats.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch_bench.json 2> $OUT/fetch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write_bench.json 2> $OUT/write.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/cfetch -o cfetch --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cfetch.out 2> $OUT/cfetch.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/cwrite -o cwrite --output-format csv -- \
    python3 $R/tools/pmc_calib.py > $OUT/cwrite.out 2> $OUT/cwrite.err
echo "exit=$?" > $OUT/done.txt
