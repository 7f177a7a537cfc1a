set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/c2shape; mkdir -p $O
for v in "32 0" "16 64" "8 128" "4 256" "16 256" "8 256"; do
  set -- $v
  if [ $2 = 0 ]; then E="PK_WAVE_LANES=$1"; else E="PK_WAVE_LANES=$1 PK_K1_BLOCK=$2"; fi
  env $E timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload config2 > $O/l$1_b$2.json 2>> $O/err.log || exit $?
done
