#!/bin/bash
# round 4: cost of fewer staged ROM banks in the 158 KB K1 (whole-handle config3 launches) — how
# much of the small-LDS kernel's loss on whole launches is its 2 banks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIBS="dual@PK_K1_SMALL=0 dual@PK_K1_SMALL=0+PK_LDS_SLOTS=2 dual@PK_K1_SMALL=0+PK_LDS_SLOTS=3" WLS="config3" STEPS=8 BENCH_EXTRA="--batches 1" tools/gpu_ab.sh r04i || exit 1
