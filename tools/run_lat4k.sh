#!/bin/bash
# lone 4,096-proof batch latency vs pass knobs (tools/pass_times.py, 5 reps each)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lat
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 100 python3 tools/pass_times.py 4096 4096 > gpurun_out/lat/$tag.log 2>&1 || { tail -5 gpurun_out/lat/$tag.log; exit 1; }
  grep -o "B=4096 wall=[0-9.]* ms" gpurun_out/lat/$tag.log | tail -1 | sed "s/^/$tag /"
}
run base FTS_X=0
run fork0 FTS_RLC_FORK=0
run work FTS_COM_FIXED_MAX=0
run lat64 FTS_LAT_BS=64
run lat128 FTS_LAT_BS=128
run base2 FTS_X=0
run fork0_2 FTS_RLC_FORK=0
