#!/bin/bash
# the driver's bench shape three times (variance of the single-burst headline)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s20x3
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --roofline-steps 2 > gpurun_out/s20x3/r$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/s20x3/r$r.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s20 run $r', round(d['value']), d['merged_batches_avg'], d['ms_per_step'])"
done
timeout -k 10 150 python3 tools/burst.py --steps 20 --reps 9 --tag gated > gpurun_out/s20x3/burst.log 2>&1 || exit 1
grep '^{' gpurun_out/s20x3/burst.log
