#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4t
timeout -k 10 200 python3 tools/transfer_profile.py 8192 > gpurun_out/c4t/tp2.log 2>&1 || { tail -20 gpurun_out/c4t/tp2.log; exit 1; }
tail -4 gpurun_out/c4t/tp2.log
bash tools/c4_sweep.sh
