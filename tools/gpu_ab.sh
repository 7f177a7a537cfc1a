#!/bin/bash
# A/B/n bench: each variant in $LIBS on each workload in $WLS, interleaved (ABAB) to spread clock
# drift; parity of the first variant's kernels when $PARITY is set.  A variant is a library name
# (pokegym_amd/lib/libpokegym_amd_<name>.so) optionally followed by @VAR=value[+VAR=value...]
# (environment settings for that run, e.g. "ilv@PK_ILV=64"; the output files use the part before
# '@' plus the values).
#
#   usage: [LIBS=...] [WLS=...] [REPS=2] [STEPS=8] [PARITY=std|<pytest -k expr>] [B64=1] bash tools/gpu_ab.sh TAG
#
# PARITY=std runs the subset every kernel change of rounds 4-6 was gated on (emulator parity + the
# benchmarked configs' flows); B64=1 adds a config3 pass on the 1 MiB (64-bank) pkbench, written to
# gpurun_out/ab_TAG64.  Round 5's per-experiment wrappers were this script with, e.g.
#   PARITY=std LIBS="diet11u diet11 diet10" WLS="config3 config4 config2" REPS=3 B64=1 ... r05m
#   PARITY=std LIBS="pre base" WLS="config3 config4 config2" REPS=3 B64=1 ... r05pre
#   LIBS="diet12 diet12@PK_K1_PRIO=1 diet12@PK_WAVE_LANES=32 diet12@PK_WAVE_LANES=64" WLS="config3 config4" ... r05shape
# (the tags and variants of every round-5 A/B are listed in profiles/r05/ab_*/summary.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-x}
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
STEPS=${STEPS:-8}
WLS=${WLS:-"config3 config4 config2"}
if [ "$PARITY" = "std" ]; then
  PARITY="copydata or warp or 64_banks or small_lds or config3_flow or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes or irq_bank or io_edges or vram_midframe"
  PARITY_FILES=${PARITY_FILES:-"tests/test_gpu_parity.py tests/test_gpu_scale.py"}
fi
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
bench_pass() {  # out_dir workloads extra_args
  local d=$1 w n
  mkdir -p $d
  for rep in $(seq 1 ${REPS:-2}); do
    for w in $2; do
      for n in $LIBS; do
        env $(runenv $n) timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --workload $w $3 > $d/${w}_$(tag $n)_$rep.json 2>> $d/err.log || return $?
      done
    done
  done
}
bench_pass $O "$WLS" "$BENCH_EXTRA" || rc=$?
if [ $rc -eq 0 ] && [ -n "$B64" ]; then
  bench_pass $R/gpurun_out/ab_${TAG}64 "config3" "--rom-banks 64" || rc=$?
fi
echo "exit=$rc" > $O/exit.txt
exit $rc
