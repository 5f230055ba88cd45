#!/bin/bash
# lanes x side-stream x HW-queue sweep of the bench (run on the GPU box)
mkdir -p gpurun_out
for q in ${QUEUES:-8 16}; do for side in ${SIDES:-1 0}; do for lanes in ${LANES:-4 6 8}; do
  r=$(GPU_MAX_HW_QUEUES=$q FTS_SIDE_STREAM=$side FTS_LANES=$lanes timeout -k 10 120 python3 bench.py --steps ${STEPS:-48} --warmup 8 --lanes $lanes --cpu-sample 0 --reuse-proofs 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']), d['ms_per_step'])") || exit 1
  echo "queues=$q side=$side lanes=$lanes -> $r" | tee -a gpurun_out/lane_sweep.txt
done; done; done
