#!/bin/bash
# A/B: bench config3 with the default library and with pokegym_amd/lib/libpokegym_amd_alt.so
# (extra environment for the B runs in $AB_ENV, e.g. "PK_WAVE_LANES=16")
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/ab
mkdir -p $O
ALT=$PWD/pokegym_amd/lib/libpokegym_amd_alt.so
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/a.json 2>&1 && \
env PK_LIB=$ALT $AB_ENV timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b.json 2>&1 && \
env PK_LIB=$ALT $AB_ENV timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "game_rom or fuzz_rom_parity and 0" > $O/b_par.log 2>&1
echo exit=$? > $O/done
