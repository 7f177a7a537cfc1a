#!/bin/bash
# round 4, second GPU call: image sub-block skew (channel aliasing) on configs[1]
# in its default and spread shapes and on configs[2]/[3]; the 78 KB-LDS K1 (two workgroups per CU,
# item 4) on configs[3]'s VecEnv flow
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIBS="cur skew256 cur@PK_WAVE_LANES=4+PK_K1_BLOCK=256 skew256@PK_WAVE_LANES=4+PK_K1_BLOCK=256 cur@PK_WAVE_LANES=8+PK_K1_BLOCK=128 skew256@PK_WAVE_LANES=8+PK_K1_BLOCK=128" WLS="config2" STEPS=8 tools/gpu_ab.sh r04b_c2 || exit 1
LIBS="cur skew256" WLS="config3" STEPS=8 tools/gpu_ab.sh r04b_c3 || exit 1
LIBS="cur skew256 lds2 lds2@PK_K1_PRIO=1" WLS="config4" STEPS=8 tools/gpu_ab.sh r04b_c4 || exit 1
