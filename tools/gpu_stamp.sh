#!/bin/bash
# K1 phase-cycle breakdown (diagnostic -DPK_STAMP build) for several workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stamp_${1:-x}; shift
mkdir -p $OUT
cd $R
rc=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}
  envs=""; args=""
  for tok in $rest; do case $tok in *=*) envs="$envs $tok";; *) args="$args $tok";; esac; done
  env $envs PK_LIB=pokegym_amd/lib/libpokegym_amd_stamp.so timeout -k 10 300 python tools/stamp_run.py $args > $OUT/$name.json 2> $OUT/$name.err || { rc=$?; break; }
done
echo "exit=$rc" > $OUT/exit.txt
