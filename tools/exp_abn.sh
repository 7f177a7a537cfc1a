#!/bin/bash
# A/B/n: bench config3 with the default library and each pokegym_amd/lib/libpokegym_amd_<name>.so
# named in $ALTS (built by pokegym_amd.build.build(out=...)); parity of the default library first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/abn
mkdir -p $O
STEPS=${STEPS:-6}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reward.py -x -q --timeout 120 --timeout-method thread > $O/par.log 2>&1 && \
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $O/main.json 2>&1 && \
for n in $ALTS; do
  env PK_LIB=$PWD/pokegym_amd/lib/libpokegym_amd_$n.so timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $O/$n.json 2>&1 || exit 1
done && \
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $O/main2.json 2>&1
echo exit=$? > $O/done
