#!/bin/bash
# bench config3 at 64 and 32 envs per wave (default library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/lanes
mkdir -p $O
PK_WAVE_LANES=64 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b64.json 2>&1 && \
PK_WAVE_LANES=32 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b32.json 2>&1
echo exit=$? > $O/done
