#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4t
timeout -k 10 200 python3 tools/transfer_profile.py 8192 > gpurun_out/c4t/tp.log 2>&1 || { tail -20 gpurun_out/c4t/tp.log; exit 1; }
tail -25 gpurun_out/c4t/tp.log
rm -rf gpurun_out/c4t/tr
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/c4t/tr -o run -- python3 bench.py --workload transfer --steps 24 --warmup 4 --cpu-sample 0 > gpurun_out/c4t/run.log 2>&1 || { tail -20 gpurun_out/c4t/run.log; exit 1; }
python3 tools/trace_share.py $(find gpurun_out/c4t/tr -name "*kernel_trace.csv" | head -1) > gpurun_out/c4t/share.txt
head -45 gpurun_out/c4t/share.txt
