#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ne8
for lib in fabric-token-sdk_amd/lib/libfts_gpu.so fabric-token-sdk_amd/lib/alt/libfts_gpu_ne8.so fabric-token-sdk_amd/lib/libfts_gpu.so fabric-token-sdk_amd/lib/alt/libfts_gpu_ne8.so; do
  FTS_LIB=$lib timeout -k 10 100 python3 tools/pass_times.py 4096 32768 81920 > gpurun_out/ne8/p.log 2>&1 || exit 1
  python3 - $lib <<'PY'
import re,sys
for line in open("gpurun_out/ne8/p.log"):
    m = re.search(r"B=(\d+) wall=([\d.]+)", line)
    nm = re.findall(r"k_rp_normalize=([\d.]+)", line)
    if m: print(sys.argv[1].split('/')[-1], "B", m.group(1), "wall", m.group(2), "normalize", nm)
PY
done
