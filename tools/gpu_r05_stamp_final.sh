#!/bin/bash
# Round-5 final kernel: phase stamps (-DPK_STAMP build, whole-handle launches; config3small = the
# small-LDS kernel the VecEnv sub-batches run) and configs[1] on the 64-bank pkbench layout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_stamp.sh r05g "config3|--workload config3" "config4|--workload config4" "config2|--workload config2" \
    "config3small|PK_K1_SMALL=1 --workload config3" && \
mkdir -p gpurun_out/rbench_r05g && \
timeout -k 10 300 python bench.py --no-cpu-baseline --workload config2 --rom-banks 64 > gpurun_out/rbench_r05g/config2_b64.json 2> gpurun_out/rbench_r05g/config2_b64.err
