#!/bin/bash
# N>1 rehearsal on one GPU: 2 ranks (gloo for the exchange, both on device 0),
# the driver's multi-GPU command shape otherwise
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dist2
FTS_DIST_BACKEND=gloo FTS_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/dist2/run.log 2>&1 || { tail -30 gpurun_out/dist2/run.log; exit 1; }
grep '^{' gpurun_out/dist2/run.log | cut -c1-400
