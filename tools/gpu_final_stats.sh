#!/bin/bash
# Round-final evidence of the driver's own command: rocprofv3 --kernel-trace --stats over exactly
# `python bench.py` (the default config3 line, CPU baseline included, as the driver runs it), so
# the committed kernel summary and the bench line's HIP-event K1 time come from one command.
# usage: bash tools/gpu_final_stats.sh TAG   (outputs in gpurun_out/fstats_TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fstats_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/stats -o stats --output-format csv -- \
    python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/err.log
echo "exit=$?" > $OUT/exit.txt
