#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4t
timeout -k 10 200 python3 tools/transfer_profile.py 8192 > gpurun_out/c4t/tp4.log 2>&1 || { tail -20 gpurun_out/c4t/tp4.log; exit 1; }
tail -3 gpurun_out/c4t/tp4.log | cut -c1-400
timeout -k 10 200 python3 -u bench.py --workload transfer --steps 64 --warmup 4 --cpu-sample 0 > gpurun_out/c4t/b.log 2>&1 || { tail -20 gpurun_out/c4t/b.log; exit 1; }
grep '^{' gpurun_out/c4t/b.log | python3 -c "import json,sys; d=json.load(sys.stdin); k=d['kernel_ms']; print(round(d['value']), d['ms_per_step'], {x: k.get(x) for x in k if x.startswith('host')})"
timeout -k 10 200 python3 -u bench.py --workload mixed --transfers 4096 --steps 32 --warmup 4 --cpu-sample 0 > gpurun_out/c4t/m.log 2>&1 || { tail -20 gpurun_out/c4t/m.log; exit 1; }
grep '^{' gpurun_out/c4t/m.log | python3 -c "import json,sys; d=json.load(sys.stdin); k=d['kernel_ms']; print(round(d['value']), d['ms_per_step'], d.get('fallback'), {x: k.get(x) for x in k if x.startswith('host')})"
