#!/bin/bash
# whole-CU K1 (158 KB LDS: every pkbench bank staged -> the ALL instance) vs the small-LDS kernel
# (2 banks, backfills a CU from the other sub-batch) for the VecEnv sub-batches: A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
LIBS="cur cur@PK_K1_SMALL=0" WLS="config3 config4 config5" STEPS=6 bash tools/gpu_ab.sh r04y || exit $?
