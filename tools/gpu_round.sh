#!/bin/bash
# one GPU session: smoke, bench, rocprof kernel-trace stats (run from the repo root)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-10} --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
