#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fork
for v in 1 0 1 0; do
  FTS_RLC_FORK=$v timeout -k 10 100 python3 tools/pass_times.py 32768 81920 > gpurun_out/fork/p.log 2>&1 || exit 1
  grep -o "B=[0-9]* wall=[0-9.]* ms" gpurun_out/fork/p.log | sed "s/^/fork$v /" | tr '\n' ' '; echo
  FTS_RLC_FORK=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --roofline-steps 2 > gpurun_out/fork/s20_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/fork/s20_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s20 fork$v', round(d['value']), d['isolated_batch']['ms'])"
done
for v in 1 0; do
  FTS_RLC_FORK=$v timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/fork/s512_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/fork/s512_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s512 fork$v', round(d['value']))"
done
