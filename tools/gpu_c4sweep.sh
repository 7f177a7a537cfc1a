set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c4sweep
mkdir -p $O
cd $R
for spec in "131072 1" "131072 2" "65536 1" "65536 2" "32768 1" "32768 2"; do
  set -- $spec
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 2 --workload config4 --envs $1 --batches $2 > $O/c4_n$1_b$2.json 2>> $O/err.log || { echo "exit=$?" > $O/exit.txt; exit 1; }
done
echo "exit=0" > $O/exit.txt
