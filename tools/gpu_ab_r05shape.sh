#!/bin/bash
# Round-5 final kernel: wave priority in the VecEnv (small-LDS) launches, and the wave width
# (32- / 64-env waves) at configs[2]'s and configs[3]'s shard sizes, re-measured after the
# instruction diet (round 4: priority -2 %, one 32-env wave per SIMD at 32,768 -7 %, one 64-env
# wave at 65,536 -12 %).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
LIBS="diet12 diet12@PK_K1_PRIO=1 diet12@PK_WAVE_LANES=32 diet12@PK_WAVE_LANES=64" WLS="config3 config4" REPS=2 STEPS=8 bash tools/gpu_ab.sh r05shape
