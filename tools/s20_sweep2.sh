#!/bin/bash
# burst (driver's 20 steps) vs pass size: larger coalesced passes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep2
run() {  # tag steps env...
  local tag=$1 steps=$2; shift 2
  env "$@" timeout -k 10 150 python3 tools/burst.py --steps $steps --reps 5 --tag "$tag" > gpurun_out/sweep2/$tag.log 2>&1 || { tail -20 gpurun_out/sweep2/$tag.log; exit 1; }
  grep '^{' gpurun_out/sweep2/$tag.log
}
run base 20 FTS_X=0
run c48k 20 FTS_COALESCE_MAX=49152
run c80k 20 FTS_COALESCE_MAX=81920
run c80k_g1000 20 FTS_COALESCE_MAX=81920 FTS_GATHER_US=1000
run c80k_l3 20 FTS_COALESCE_MAX=81920 FTS_LANES=3
run base_s64 64 FTS_X=0
run c80k_s64 64 FTS_COALESCE_MAX=81920
