#!/bin/bash
# FTS_RLC_FORK A/B on the action-level workloads (request, mixed), alternating on one box
set -o pipefail
OUT=gpurun_out/fka
mkdir -p $OUT
run() {  # tag fork args...
  local tag=$1 fk=$2; shift 2
  FTS_RLC_FORK=$fk timeout -k 10 240 python3 bench.py --cpu-sample 0 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  grep '^{' $OUT/$tag.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$tag', round(d['value']), d['ms_per_step'])"
}
for r in 1 2; do
  run req_f1_$r 1 --workload request --steps 96 --warmup 4
  run req_f2_$r 2 --workload request --steps 96 --warmup 4
  run mix_f1_$r 1 --workload mixed --transfers 4096 --steps 48 --warmup 4
  run mix_f2_$r 2 --workload mixed --transfers 4096 --steps 48 --warmup 4
done
