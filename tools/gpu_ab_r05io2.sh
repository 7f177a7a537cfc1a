#!/bin/bash
# A/B of the IO read served by the common path's image load (libpokegym_amd_diet13: the rare IO read
# needs no memory round trip of its own) against the final kernel (diet12), parity subset of
# diet13 first; then tools/gpu_ab_r05shape.sh (priority / wave width on the final kernel).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram or watchdog or instr_count or wave_shapes" LIBS="diet13 diet12" WLS="config3 config4 config2" REPS=2 STEPS=8 bash tools/gpu_ab.sh r05n && \
LIBS="diet13 diet12" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05n64 && \
bash tools/gpu_ab_r05shape.sh
