#!/bin/bash
# A/B of the rare IO read with DIV served first, on its own (libpokegym_amd_diet15)
# against the final kernel (diet12); parity subset of diet15 first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet15 diet12" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05p && \
LIBS="diet15 diet12" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05p64
