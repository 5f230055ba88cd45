#!/bin/bash
# A/B of library builds on the GPU box: isolated per-kernel times (one lane)
# and the pipelined bench, for each .so given in LIBS (default: in-tree lib).
#   LIBS="fabric-token-sdk_amd/lib/ab/head.so fabric-token-sdk_amd/lib/libfts_gpu.so" bash tools/ab.sh
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-fabric-token-sdk_amd/lib/libfts_gpu.so}
for lib in $LIBS; do
  echo "== $lib"
  FTS_LIB=$lib TAG=$(basename $lib) timeout -k 10 120 python3 tools/kernel_times.py 4096 5 || exit 1
  for ln in ${BENCH_LANES:-8}; do
    r=$(FTS_LIB=$lib timeout -k 10 150 python3 bench.py --steps ${STEPS:-64} --warmup 8 --lanes $ln --distinct 1 --cpu-sample 0 --roofline-steps 1 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']), d['ms_per_step'])") || exit 1
    echo "bench lanes=$ln -> $r"
  done
done
