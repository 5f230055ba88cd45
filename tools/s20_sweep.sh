#!/bin/bash
# A/B of the library's coalescing knobs on the driver's 20-step burst (tools/burst.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 tools/burst.py --steps ${STEPS:-20} --reps 7 --tag "$tag" > gpurun_out/sweep/$tag.log 2>&1 || { tail -20 gpurun_out/sweep/$tag.log; exit 1; }
  grep '^{' gpurun_out/sweep/$tag.log
}
run base FTS_X=0
run c16k FTS_COALESCE_MAX=16384
run c12k FTS_COALESCE_MAX=12288
run c8k FTS_COALESCE_MAX=8192

run l8c16k FTS_LANES=8 FTS_COALESCE_MAX=16384

run g0 FTS_GATHER_US=0
run cf0 FTS_COM_FIXED_MAX=0
run cf32k FTS_COM_FIXED_MAX=32768

