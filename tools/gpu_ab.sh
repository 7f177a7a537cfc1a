#!/bin/bash
# A/B/n bench: each pokegym_amd/lib/libpokegym_amd_<name>.so in $LIBS on each workload in $WLS,
# interleaved (ABAB) to spread clock drift; parity of the first library's kernels when $PARITY is set.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/ab_${1:-x}
mkdir -p $O
STEPS=${STEPS:-8}
rc=0
if [ -n "$PARITY" ]; then
  n=${LIBS%% *}
  env PK_LIB=$R/pokegym_amd/lib/libpokegym_amd_$n.so timeout -k 10 600 python -u -m pytest ${PARITY_FILES:-tests/test_gpu_parity.py} -x -q --timeout 200 --timeout-method thread -k "$PARITY" > $O/par_$n.log 2>&1 || { rc=$?; echo "exit=$rc" > $O/exit.txt; exit $rc; }
fi
for rep in 1 2; do
  for w in $WLS; do
    for n in $LIBS; do
      env PK_LIB=$R/pokegym_amd/lib/libpokegym_amd_$n.so timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --workload $w $BENCH_EXTRA > $O/${w}_${n}_$rep.json 2>> $O/err.log || { rc=$?; break 3; }
    done
  done
done
echo "exit=$rc" > $O/exit.txt
