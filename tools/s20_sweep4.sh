#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep4
run() {  # tag steps env...
  local tag=$1 steps=$2; shift 2
  env "$@" timeout -k 10 150 python3 tools/burst.py --steps $steps --reps 9 --tag "$tag" > gpurun_out/sweep4/$tag.log 2>&1 || { tail -20 gpurun_out/sweep4/$tag.log; exit 1; }
  grep '^{' gpurun_out/sweep4/$tag.log
}
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --roofline-steps 2 > gpurun_out/sweep4/b_$tag.log 2>&1 || { tail -20 gpurun_out/sweep4/b_$tag.log; exit 1; }
  grep '^{' gpurun_out/sweep4/b_$tag.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench512 $tag', round(d['value']), d['merged_batches_avg'], d['isolated_batch']['ms'])"
}
run base 20 FTS_X=0
run l4 20 FTS_LANES=4
run c80k_g1000_l4 20 FTS_COALESCE_MAX=81920 FTS_GATHER_US=1000 FTS_LANES=4
run c80k_g1000_l3 20 FTS_COALESCE_MAX=81920 FTS_GATHER_US=1000 FTS_LANES=3
run c64k_g1000_l4 20 FTS_COALESCE_MAX=65536 FTS_GATHER_US=1000 FTS_LANES=4
run c96k_g1000_l4 20 FTS_COALESCE_MAX=98304 FTS_GATHER_US=1000 FTS_LANES=4
run c80k_g500_l4 20 FTS_COALESCE_MAX=81920 FTS_GATHER_US=500 FTS_LANES=4
bench c80k_g1000_l4 FTS_COALESCE_MAX=81920 FTS_GATHER_US=1000 FTS_LANES=4
bench c80k_g1000_l3 FTS_COALESCE_MAX=81920 FTS_GATHER_US=1000 FTS_LANES=3
