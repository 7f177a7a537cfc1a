#!/bin/bash
# A/B of the rare IO read with JOYP served second (libpokegym_amd_diet16) against DIV-first alone
# (diet15) and the final kernel of the diet (diet12); parity subset of diet16 first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet16 diet15 diet12" WLS="config3 config4 config2" REPS=2 STEPS=8 bash tools/gpu_ab.sh r05q && \
LIBS="diet16 diet15 diet12" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05q64
