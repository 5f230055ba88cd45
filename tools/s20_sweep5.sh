#!/bin/bash
# burst A/B with the bench's 16 hardware queues; old defaults vs new
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep5
run() {  # tag steps env...
  local tag=$1 steps=$2; shift 2
  env "$@" timeout -k 10 150 python3 tools/burst.py --steps $steps --reps 9 --tag "$tag" > gpurun_out/sweep5/$tag.log 2>&1 || { tail -20 gpurun_out/sweep5/$tag.log; exit 1; }
  grep '^{' gpurun_out/sweep5/$tag.log
}
run old 20 FTS_LANES=5 FTS_COALESCE_MAX=32768 FTS_GATHER_US=300
run new 20 FTS_X=0
run new_l5 20 FTS_LANES=5
run new_l3 20 FTS_LANES=3
run new_l6 20 FTS_LANES=6
run new_g2000 20 FTS_GATHER_US=2000
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/sweep5/b20.log 2>&1 || exit 1
grep '^{' gpurun_out/sweep5/b20.log | cut -c1-300
