#!/bin/bash
# FP256BN GLV nym chain: idemix GPU tests, then the FP256BN workload
set -o pipefail
OUT=gpurun_out/fglv
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_idemix.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -2 $OUT/pt.log
timeout -k 10 240 python3 bench.py --workload idemix --idemix-curve fp256bn --steps 32 --warmup 4 > $OUT/fbn.log 2>&1 || { tail -5 $OUT/fbn.log; exit 1; }
grep '^{' $OUT/fbn.log | tail -1 > $OUT/fbn.json
python3 -c "import json; d=json.load(open('$OUT/fbn.json')); print(round(d['value']), d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 240 python3 bench.py --workload idemix --idemix-curve fp256bn --steps 32 --warmup 4 --msg-len 64 --cpu-sample 0 > $OUT/fbn64.log 2>&1 || { tail -5 $OUT/fbn64.log; exit 1; }
grep '^{' $OUT/fbn64.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('L64', round(d['value']), d['roofline']['kernel_ms'])"
