set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PARITY_FILES="tests/test_gpu_parity.py tests/test_gpu_scale.py" PARITY="copydata or warp or 64_banks or small_lds or config4_flow or config5_flow or fuzz_rom_parity or hram or watchdog" LIBS="bf base nobf" WLS="config3 config4 config2" REPS=2 STEPS=8 bash tools/gpu_ab.sh r05w && \
LIBS="bf base" WLS="config3" REPS=2 STEPS=8 BENCH_EXTRA="--rom-banks 64" bash tools/gpu_ab.sh r05w64
