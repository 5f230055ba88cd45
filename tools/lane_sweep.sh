#!/bin/bash
# device lanes x coalescing cap x in-flight batches sweep of the bench (GPU box)
mkdir -p gpurun_out
for lanes in ${LANES:-2 4 8}; do for cm in ${CMAX:-4096 16384 32768}; do for inf in ${INFLIGHT:-16}; do
  r=$(FTS_COALESCE_MAX=$cm timeout -k 10 150 python3 bench.py --steps ${STEPS:-96} --warmup 16 --lanes $lanes --inflight $inf --distinct 1 --cpu-sample 0 --roofline-steps 1 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']), d['ms_per_step'], d['merged_batches_avg'])") || exit 1
  echo "lanes=$lanes coalesce_max=$cm inflight=$inf -> $r" | tee -a gpurun_out/lane_sweep.txt
done; done; done
