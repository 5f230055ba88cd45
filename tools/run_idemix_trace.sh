#!/bin/bash
# kernel + memory-copy timeline of the idemix workload (3 calls in flight)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/idtr
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT -o run -- python3 bench.py --workload idemix --steps 16 --warmup 2 --cpu-sample 0 > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
grep '^{' $OUT/log | tail -1 | cut -c1-200
find $OUT -name "*.csv" | xargs ls -la
