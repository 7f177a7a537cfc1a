#!/bin/bash
# config2 (4,096 envs): two narrower waves per SIMD with the priority variant vs one 32-env wave
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/c2shape
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 2 --no-cpu-baseline > $O/default_$rep.json 2>> $O/err.log || exit 1
  env PK_WAVE_LANES=16 PK_K1_BLOCK=512 timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 2 --no-cpu-baseline > $O/l16b512_$rep.json 2>> $O/err.log || exit 1
  env PK_WAVE_LANES=8 PK_K1_BLOCK=512 timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 2 --no-cpu-baseline > $O/l8b512_$rep.json 2>> $O/err.log || exit 1
done
echo exit=0 > $O/exit.txt
