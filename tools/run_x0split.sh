#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/x0s
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_scale.py tests/test_gpu_actions.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x0s/pt.log 2>&1 || { tail -30 gpurun_out/x0s/pt.log; exit 1; }
tail -2 gpurun_out/x0s/pt.log
for v in 0 1; do
  FTS_X0_SPLIT=$v timeout -k 10 150 python3 tools/burst.py --steps 20 --reps 9 --tag split$v > gpurun_out/x0s/b$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/x0s/b$v.log
  FTS_X0_SPLIT=$v timeout -k 10 100 python3 tools/pass_times.py 4096 32768 81920 > gpurun_out/x0s/p$v.log 2>&1 || exit 1
  cut -c1-60 gpurun_out/x0s/p$v.log
done
for v in 0 1; do
  FTS_X0_SPLIT=$v timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/x0s/s$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/x0s/s$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench512 split$v', round(d['value']), d['merged_batches_avg'], d['isolated_batch']['ms'], d['isolated_pass'])"
done
