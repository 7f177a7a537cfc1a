#!/bin/bash
# wave-priority A/B: placements on config3 (65,536 envs), the templated product library (tpl) on
# config4/config2 (one wave per SIMD: no priority variant) and at 131,072 envs; tpl parity first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIBS="tpl" WLS="config3" PARITY="512_thread or game_rom" bash tools/gpu_ab.sh prio2 || exit 1
LIBS="head prio1 prio3 prio5" WLS="config3" bash tools/gpu_ab.sh prio2 || exit 1
LIBS="head tpl" WLS="config4 config2" bash tools/gpu_ab.sh prio2_c4 || exit 1
LIBS="head tpl" WLS="config3" BENCH_EXTRA="--envs 131072" bash tools/gpu_ab.sh prio2_131k
