#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cbs
FTS_CHAIN_BS=256 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cbs/pt.log 2>&1 || { tail -30 gpurun_out/cbs/pt.log; exit 1; }
tail -1 gpurun_out/cbs/pt.log
for v in 64 256 64 256; do
  FTS_CHAIN_BS=$v timeout -k 10 100 python3 tools/pass_times.py 32768 81920 > gpurun_out/cbs/p.log 2>&1 || exit 1
  python3 - $v <<'PY'
import re,sys
for line in open("gpurun_out/cbs/p.log"):
    m = re.search(r"B=(\d+) wall=([\d.]+)", line)
    cv = re.findall(r"k_rp_com_var=([\d.]+)", line); hj = re.findall(r"k_rp_hsum_join=([\d.]+)", line)
    if m: print("bs", sys.argv[1], "B", m.group(1), "wall", m.group(2), "com_var", cv, "hsum_join", hj)
PY
done
for v in 64 256; do
  FTS_CHAIN_BS=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --roofline-steps 2 > gpurun_out/cbs/s20_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/cbs/s20_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s20 bs$v', round(d['value']))"
  FTS_CHAIN_BS=$v timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/cbs/s512_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/cbs/s512_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('s512 bs$v', round(d['value']))"
done
