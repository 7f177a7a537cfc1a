#!/bin/bash
# K1 experiment session: GPU parity, then bench config3 at 64/32 lanes per wave and config2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/exp1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/par.log 2>&1 && \
PK_WAVE_LANES=64 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b64.json 2>&1 && \
PK_WAVE_LANES=32 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b32.json 2>&1 && \
timeout -k 10 300 python bench.py --workload config2 --envs 4096 --steps 4 --warmup 1 --no-cpu-baseline > $O/c2.json 2>&1
echo exit=$? > $O/done
