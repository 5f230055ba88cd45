#!/bin/bash
# kernel timelines of one isolated pass (4,096 and 32,768 proofs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/trace
for B in 4096 32768; do
  rm -rf gpurun_out/trace/p$B
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace/p$B -o run -- python3 tools/pass_times.py $B > gpurun_out/trace/p$B.log 2>&1 || { tail -20 gpurun_out/trace/p$B.log; exit 1; }
  tail -1 gpurun_out/trace/p$B.log | cut -c1-300
  python3 tools/trace_pass.py $(find gpurun_out/trace/p$B -name "*kernel_trace.csv" | head -1) k_rp_decode > gpurun_out/trace/timeline_$B.txt
  head -60 gpurun_out/trace/timeline_$B.txt
done
