#!/bin/bash
# A/B of the operand preload (PK_PRE: the next address formed and its operand requested at the end of
# the iteration; libpokegym_amd_pre) against the committed kernel (base); parity subset of pre first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="pre base" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05pre && \
LIBS="pre base" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05pre64
