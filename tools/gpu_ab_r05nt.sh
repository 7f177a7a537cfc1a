#!/bin/bash
# A/B of non-temporal VRAM stores in K1 (libpokegym_amd_ntv, -DPK_NT_VRAM=1) against the committed kernel
# (base), parity subset of ntv first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or fuzz_rom_parity or hram" LIBS="ntv base" WLS="config3 config4 config2" REPS=3 STEPS=8 bash tools/gpu_ab.sh r05nt
