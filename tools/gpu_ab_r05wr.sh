#!/bin/bash
# A/B of the slow write path with sound-register and joypad-select writes served first, each on its
# own (libpokegym_amd_diet17) against the final kernel (diet16); parity subset of diet17 first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet17 diet16" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05r && \
LIBS="diet17 diet16" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05r64
