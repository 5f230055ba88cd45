#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fxo
FTS_FX_ORDER=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fxo/pt.log 2>&1 || { tail -30 gpurun_out/fxo/pt.log; exit 1; }
tail -1 gpurun_out/fxo/pt.log
for v in 0 1 0 1; do
  FTS_FX_ORDER=$v timeout -k 10 100 python3 tools/pass_times.py 32768 81920 > gpurun_out/fxo/p$v.log 2>&1 || exit 1
  python3 - $v <<'PY'
import re,sys
for line in open("gpurun_out/fxo/p%s.log" % sys.argv[1]):
    m = re.search(r"B=(\d+) wall=([\d.]+).*k_rp_fixed_exact=([\d.]+)", line)
    if m: print("order", sys.argv[1], "B", m.group(1), "wall", m.group(2), "fixed_exact", m.group(3))
PY
done
for v in 0 1; do
  FTS_FX_ORDER=$v timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/fxo/s$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/fxo/s$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench512 order$v', round(d['value']), d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
