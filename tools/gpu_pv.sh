#!/bin/bash
# after the three-level priority schedule: parity of the wide shapes + the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/pv_final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -k "512_thread or game_rom or hram or 64_banks or geometry or shard" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench.err && \
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > $O/bench_config4.json 2>> $O/bench.err && \
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > $O/bench_config5.json 2>> $O/bench.err
echo "exit=$?" > $O/exit.txt
