#!/bin/bash
# PCIe-inclusive rate: config3 / config5 with every step's obs handed to pinned host buffers
# (bench.py --host-obs), next to the device-resident lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/hostobs
mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/config3.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-obs > $O/config3_hostobs.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $O/config5.json 2>> $O/err.log && \
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline --host-obs > $O/config5_hostobs.json 2>> $O/err.log
echo "exit=$?" > $O/exit.txt
