#!/bin/bash
# round 4: configs[3]'s per-GPU shard sizes (N = 1, 2, 4, 8: 262,144 / 131,072 / 65,536 / 32,768 envs
# per GPU) through VecEnv with the round-4 defaults, and the 131,072 shard with 32-env waves in the
# small-LDS kernel (sub-batches backfill each other's freed workgroup slots)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for e in 262144 131072 65536 32768; do
  LIBS="dual" WLS="config4" STEPS=10 BENCH_EXTRA="--envs $e" tools/gpu_ab.sh r04g_e$e || exit 1
done
LIBS="dual@PK_WAVE_LANES=32+PK_K1_SMALL=1" WLS="config4" STEPS=10 BENCH_EXTRA="--envs 131072" tools/gpu_ab.sh r04g_e131072s || exit 1
