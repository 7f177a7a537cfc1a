#!/bin/bash
# round 4: GPU parity suite on the dual-K1 library (all but the 10k-step horizon file), then the
# small-LDS kernel's bench A/B on configs[3]'s N=8 and N=4 shards
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TESTS=tests PYTEST_EXTRA="--ignore=tests/test_gpu_horizon.py --durations=25" PYTEST_LIMIT=900 bash tools/gpu_tests.sh r04d || exit 1
grep -q "exit=0" gpurun_out/tests_r04d/exit.txt || exit 1
cp pokegym_amd/lib/libpokegym_amd.so pokegym_amd/lib/libpokegym_amd_dual.so
LIBS="dual dual@PK_K1_SMALL=0" WLS="config4" STEPS=8 tools/gpu_ab.sh r04d_c4 || exit 1
LIBS="dual dual@PK_K1_SMALL=0" WLS="config4" STEPS=8 BENCH_EXTRA="--envs 65536" tools/gpu_ab.sh r04d_c4_65k || exit 1
