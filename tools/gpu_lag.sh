set -o pipefail
mkdir -p gpurun_out
PARITY="512_thread or warp or hram" LIBS="lag base" WLS="config4 config3" STEPS=8 tools/gpu_ab.sh lag1 && tools/gpu_wavetime.sh r03wl config4 && PK_LIB=pokegym_amd/lib/libpokegym_amd_wtlag.so timeout -k 10 240 python -u tools/wavetime_run.py --workload config4 > gpurun_out/wt_r03wl/config4_lag.json 2>/dev/null
