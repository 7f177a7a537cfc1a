#!/bin/bash
# (a) the 32,768-env shard as two 16-env waves per SIMD (wide shape -> wave-priority variant) vs
#     the default one 32-env wave per SIMD; (b) round profiles of the final kernel (tools/gpu_round_prof.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/l16
mkdir -p $O
for w in config4 config5; do
  timeout -k 10 300 python bench.py --workload $w --steps 8 --warmup 2 --no-cpu-baseline > $O/${w}_default.json 2>> $O/err.log || exit 1
  env PK_WAVE_LANES=16 PK_K1_BLOCK=512 timeout -k 10 300 python bench.py --workload $w --steps 8 --warmup 2 --no-cpu-baseline > $O/${w}_l16b512.json 2>> $O/err.log || exit 1
done
bash tools/gpu_round_prof.sh r02p "config3|" "config2|--workload config2" "config4|--workload config4" "config5|--workload config5" "config3_b64|--rom-banks 64"
