#!/bin/bash
# per-wave K1 timing (diagnostic -DPK_WAVETIME build) for the given workloads
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/wt_${1:-x}; shift
mkdir -p $OUT
cd $R
rc=0
for w in "$@"; do
  PK_LIB=pokegym_amd/lib/libpokegym_amd_wt.so timeout -k 10 240 python -u tools/wavetime_run.py --workload $w --out $OUT/$w.npz > $OUT/$w.json 2> $OUT/$w.err || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
exit $rc
