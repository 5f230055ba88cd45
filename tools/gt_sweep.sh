#!/bin/bash
# C5 (1 % tampered) fallback cost vs group-test parameters, plus the GPU group-test test
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt/pt.log 2>&1 || { tail -30 gpurun_out/gt/pt.log; exit 1; }
tail -1 gpurun_out/gt/pt.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --workload mixed --transfers 4096 --steps 32 --warmup 4 --cpu-sample 0 > gpurun_out/gt/$tag.log 2>&1 || { tail -20 gpurun_out/gt/$tag.log; exit 1; }
  grep '^{' gpurun_out/gt/$tag.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$tag', round(d['value']), d['ms_per_step'], d.get('fallback'))"
}
run base FTS_X=0
run g128 FTS_GT1=128 FTS_GT2_MIN=4096
run g256 FTS_GT1=256 FTS_GT2_MIN=4096
run g256_8k FTS_GT1=256 FTS_GT2_MIN=8192
run g64_0 FTS_GT1=64 FTS_GT2_MIN=0
