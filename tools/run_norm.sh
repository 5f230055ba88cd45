#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/norm
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/norm/smoke.log 2>&1 || { tail -20 gpurun_out/norm/smoke.log; exit 1; }
tail -1 gpurun_out/norm/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/norm/pt.log 2>&1 || { tail -30 gpurun_out/norm/pt.log; exit 1; }
tail -1 gpurun_out/norm/pt.log
timeout -k 10 100 python3 tools/pass_times.py 4096 32768 81920 > gpurun_out/norm/p.log 2>&1 || exit 1
python3 - <<'PY'
import re
for line in open("gpurun_out/norm/p.log"):
    m = re.search(r"B=(\d+) wall=([\d.]+)", line)
    nm = re.findall(r"k_rp_normalize=([\d.]+)", line)
    if m: print("B", m.group(1), "wall", m.group(2), "normalize", nm)
PY
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --roofline-steps 2 > gpurun_out/norm/s20_$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/norm/s20_$r.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s20', round(d['value']), d['merged_batches_avg'], d['roofline']['kernel_ms'], d['isolated_batch']['ms'])"
done
timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/norm/s512.log 2>&1 || exit 1
grep '^{' gpurun_out/norm/s512.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s512', round(d['value']), d['merged_batches_avg'], d['isolated_pass'])"
