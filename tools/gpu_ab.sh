#!/bin/bash
# A/B/n bench: each variant in $LIBS on each workload in $WLS, interleaved (ABAB) to spread clock
# drift; parity of the first variant's kernels when $PARITY is set.  A variant is a library name
# (pokegym_amd/lib/libpokegym_amd_<name>.so) optionally followed by @VAR=value[+VAR=value...]
# (environment settings for that run, e.g. "ilv@PK_ILV=64"; the output files use the part before
# '@' plus the values).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/ab_${1:-x}
mkdir -p $O
STEPS=${STEPS:-8}
rc=0
runenv() {  # variant -> "PK_LIB=... [VAR=value]"
  local n=${1%%@*} e=""
  [[ $1 == *@* ]] && e=${1#*@} && e=${e//+/ }
  echo "PK_LIB=$R/pokegym_amd/lib/libpokegym_amd_$n.so $e"
}
tag() { local t=${1//@/_}; t=${t//+/_}; echo ${t//=/}; }
if [ -n "$PARITY" ]; then
  n=${LIBS%% *}
  env $(runenv $n) timeout -k 10 600 python -u -m pytest ${PARITY_FILES:-tests/test_gpu_parity.py} -x -q --timeout 200 --timeout-method thread -k "$PARITY" > $O/par_$(tag $n).log 2>&1 || { rc=$?; echo "exit=$rc" > $O/exit.txt; exit $rc; }
fi
for rep in $(seq 1 ${REPS:-2}); do
  for w in $WLS; do
    for n in $LIBS; do
      env $(runenv $n) timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --workload $w $BENCH_EXTRA > $O/${w}_$(tag $n)_$rep.json 2>> $O/err.log || { rc=$?; break 3; }
    done
  done
done
echo "exit=$rc" > $O/exit.txt
