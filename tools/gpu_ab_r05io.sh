#!/bin/bash
# A/B of the DIV/JOYP common-path read (libpokegym_amd_io), + the sound-write bypass (io2), against the committed kernel (base), with the
# parity subset of the io library first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="io2 io base" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05io
