#!/bin/bash
# final check of the shipped defaults: smoke, every GPU test, the driver's bench line,
# the lone-batch latency, and rocprofv3 stats of the driver's bench command
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('driver-shape', round(d['value']), d['roofline']['frac'], d['roofline']['traffic'], d['isolated_batch']['ms'])"
timeout -k 10 100 python3 tools/pass_times.py 4096 4096 > $OUT/lat.log 2>&1 || exit 1
grep -o "B=4096 wall=[0-9.]* ms" $OUT/lat.log
rm -rf $OUT/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 6 $OUT/prof/isolated.json
