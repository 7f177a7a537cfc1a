#!/bin/bash
# A/B of the round-5 instruction diet (DAA in the rare read block, the prefetch flag folded into a
# pbytes sentinel, cycle counts in the microcode V word; libpokegym_amd_diet) against the committed
# kernel (base); parity subset of diet first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet11u diet11 diet10" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05m && \
LIBS="diet11u diet11 diet10" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05m64
