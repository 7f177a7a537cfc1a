#!/bin/bash
# throughput vs envs per GPU on the final kernel (the N=2 / N=4 shard shapes of configs[3])
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/envs_final
mkdir -p $O
timeout -k 10 300 python bench.py --envs 131072 --steps 6 --warmup 2 --no-cpu-baseline > $O/config3_n131072.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --envs 262144 --steps 4 --warmup 1 --no-cpu-baseline > $O/config3_n262144.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --workload config4 --envs 131072 --steps 6 --warmup 2 --no-cpu-baseline > $O/config4_n131072.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --workload config4 --envs 65536 --steps 6 --warmup 2 --no-cpu-baseline > $O/config4_n65536.json 2>> $O/err.log
echo "exit=$?" > $O/exit.txt
