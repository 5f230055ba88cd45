#!/bin/bash
# idemix nym-signature workload: bench line + rocprofv3 kernel stats of the same command
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/idemix
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --workload idemix --steps 32 --warmup 4 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; cut -c1-900 $OUT/bench.json
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof -o run -- python3 bench.py --workload idemix --steps 16 --warmup 2 --cpu-sample 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -5 $OUT/kernel_stats.csv
