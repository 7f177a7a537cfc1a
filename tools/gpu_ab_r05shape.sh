#!/bin/bash
# Round-5 final kernel: wave priority in the VecEnv (small-LDS) launches and 64-env waves at
# configs[2]'s 65,536 envs, re-measured after the instruction diet (round 4: -2 % / -12 %).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
LIBS="diet12 diet12@PK_K1_PRIO=1 diet12@PK_WAVE_LANES=64" WLS="config3 config4" REPS=2 STEPS=8 bash tools/gpu_ab.sh r05shape
