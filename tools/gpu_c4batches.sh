set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/c4batches; mkdir -p $O
for rep in 1 2; do
for b in 1 2 4; do timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload config4 --batches $b > $O/b${b}_$rep.json 2>>$O/err.log || exit $?; done
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload config3 --envs 32768 > $O/raw32k_$rep.json 2>>$O/err.log || exit $?
done
