#!/bin/bash
# A/B of the slow write path with sound-register and joypad-select writes served first, each on its
# own (+ ROM bank writes: libpokegym_amd_diet18) against the previous step (diet17); parity subset of diet18 first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet18 diet17" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05s && \
LIBS="diet18 diet17" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05s64
