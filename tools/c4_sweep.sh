#!/bin/bash
# C4 transfer workload: in-flight calls / lanes A/B (one process per setting)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python3 -u bench.py --workload transfer --steps 64 --warmup 4 --cpu-sample 0 "$@" > gpurun_out/c4/$tag.log 2>&1 || { tail -20 gpurun_out/c4/$tag.log; exit 1; }
  grep '^{' gpurun_out/c4/$tag.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); k=d['kernel_ms']; print('$tag', round(d['value']), d['ms_per_step'], 'parse', k.get('host_parse'), 'stage', k.get('host_stage'), 'com_var', k.get('k_rp_com_var'))"
}
run if3 --action-inflight 3
run if4 --action-inflight 4
run if5 --action-inflight 5

run t16k_if3 --action-inflight 3 --transfers 16384
