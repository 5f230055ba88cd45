#!/bin/bash
# Quick GPU iteration: gpu tests -> isolated kernel times -> pipelined bench
# (device lanes in BENCH_LANES) -> optional kernel trace (TRACE=1) of the
# pipelined bench.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 120 python3 tools/kernel_times.py ${KT_B:-4096} 5 || exit 1
for ln in ${BENCH_LANES:-2}; do
  r=$(timeout -k 10 150 python3 bench.py --steps ${STEPS:-96} --warmup 16 --lanes $ln --distinct 1 --cpu-sample 0 --roofline-steps 1 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']), d['ms_per_step'], d['merged_batches_avg'])") || exit 1
  echo "bench lanes=$ln -> $r"
done
if [ "${TRACE:-0}" = 1 ]; then
  rm -rf gpurun_out/trace
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace -o run -- python3 bench.py --steps 64 --warmup 16 --lanes ${TRACE_LANES:-2} --distinct 1 --cpu-sample 0 --roofline-steps 1 > gpurun_out/trace.log 2>&1 || exit 1
fi
