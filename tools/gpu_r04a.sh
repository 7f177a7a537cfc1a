#!/bin/bash
# round 4, first GPU call: K1 wave-shape re-sweep on the round-3 kernel (one wave per SIMD at the
# benchmarked env counts vs two), the single-env configs[0] shape, and the driver's default bench
# under rocprofv3 with the fork-free CPU baseline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r04a
mkdir -p $O
LIBS="cur cur@PK_WAVE_LANES=32" WLS="config4 config5" STEPS=8 tools/gpu_ab.sh r04a_c4 || exit 1
LIBS="cur cur@PK_WAVE_LANES=64" WLS="config3" STEPS=8 tools/gpu_ab.sh r04a_c3 || exit 1
timeout -k 10 300 python bench.py --workload config1 --steps 200 --warmup 20 > $O/config1.json 2> $O/config1.err || exit 1
bash tools/gpu_final_stats.sh r04a
cd $R && timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_scale.py::test_config4_flow_vs_oracle_per_env tests/test_gpu_reward.py::test_gpu_reward_replay_at_scale > $O/pytest_new.log 2>&1
echo "pytest exit=$?" >> $O/pytest_new.log
