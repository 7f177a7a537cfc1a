#!/bin/bash
# Rehearse bench.py's multi-rank flow (torchrun, 2 ranks, config4 default, barriers, max-over-ranks
# timing, one JSON line) on a one-GPU box: both ranks on device 0 over gloo (PK_BENCH_REHEARSAL);
# 32,768 envs per rank is the N=8 per-GPU shard shape (16-env waves).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rehearse
mkdir -p $OUT
cd $R
PK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --envs 32768 \
    > $OUT/n2_32768.json 2> $OUT/n2_32768.err && \
PK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 \
    > $OUT/n2_default.json 2> $OUT/n2_default.err && \
PK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 4 --warmup 1 --workload config5 --envs 16384 \
    > $OUT/n2_config5.json 2> $OUT/n2_config5.err
echo "exit=$?" > $OUT/exit.txt
