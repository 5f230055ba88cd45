#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/idemix2
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_idemix.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1; rc=$?; tail -15 $OUT/pt.log; [ $rc -eq 0 ] || exit 1
for c in bn254 fp256bn; do
  timeout -k 10 300 python3 -u bench.py --workload idemix --idemix-curve $c --steps 32 --warmup 4 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  grep '^{' $OUT/bench_$c.log | tail -1 > $OUT/bench_$c.json; cut -c1-400 $OUT/bench_$c.json
done
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof -o run -- python3 bench.py --workload idemix --idemix-curve fp256bn --steps 16 --warmup 2 --cpu-sample 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_fbn.csv \;
head -5 $OUT/kernel_stats_fbn.csv
