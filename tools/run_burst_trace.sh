#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/btrace
rm -rf gpurun_out/btrace/tr
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/btrace/tr -o run -- python3 tools/burst.py --steps 20 --reps 2 > gpurun_out/btrace/run.log 2>&1 || { tail -20 gpurun_out/btrace/run.log; exit 1; }
python3 tools/burst_timeline.py $(find gpurun_out/btrace/tr -name "*kernel_trace.csv" | head -1) 250 > gpurun_out/btrace/timeline.txt
cat gpurun_out/btrace/timeline.txt
