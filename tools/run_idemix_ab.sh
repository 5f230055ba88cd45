#!/bin/bash
# idemix throughput breakdown: calls in flight, batch size and message length
set -o pipefail
OUT=gpurun_out/idab
mkdir -p $OUT
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --workload idemix --steps 32 --warmup 4 --cpu-sample 0 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  grep '^{' $OUT/$tag.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$tag', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run if1 --action-inflight 1
run if3 --action-inflight 3
run if6 --action-inflight 6
run L64 --msg-len 64
run big --sigs 262144
run fbn --idemix-curve fp256bn
run fbnL64 --idemix-curve fp256bn --msg-len 64
