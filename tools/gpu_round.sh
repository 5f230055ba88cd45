#!/bin/bash
# One GPU session (run from the repo root on the gpurun box):
#   smoke -> [pytest -m gpu] -> bench -> INT-peak microbench -> rocprofv3
#   kernel-trace stats (CSV) -> PMC passes (one counter group per run).
# Every GPU step has its own time limit; the first failure ends the script.
# Env: STEPS (bench steps), TESTS=1 (run pytest -m gpu), PMC=0 (skip counters),
#      EXTRA=0 (skip the action-level benches), TAG (suffix of the output directory names).
set -o pipefail
TAG=${TAG:-r01}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -30 $OUT/$name.log; exit 1; fi
}
step smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()"
if [ "${TESTS:-0}" = 1 ]; then
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  tail -3 $OUT/pytest_gpu.log
fi
step bench 400 python3 -u bench.py --steps ${STEPS:-512} --warmup 64
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
cat $OUT/bench.json
step int_peak 120 fabric-token-sdk_amd/lib/int_peak
cat $OUT/int_peak.log
rm -rf $OUT/prof_$TAG
step rocprof 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 256 --warmup 64 --distinct 1 --roofline-steps 6 --pass-batches 8 --cpu-sample 0
grep '^{' $OUT/rocprof.log | tail -1 > $OUT/bench_rocprof.json
python3 tools/prof_summary.py $(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1) 6 $OUT/prof_$TAG/isolated.json
if [ "${PMC:-1}" = 1 ]; then
  # separate passes (TCC: FETCH_SIZE uses 3 slots, WRITE_SIZE 2)
  PB="python3 bench.py --steps 4 --warmup 4 --inflight 4 --distinct 1 --roofline-steps 2 --pass-batches 8 --cpu-sample 0"
  step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_fetch_$TAG -o run -- $PB
  step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_write_$TAG -o run -- $PB
  step pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmc_valu_$TAG -o run -- $PB
  python3 tools/pmc_summary.py $OUT $TAG $OUT/traffic_$TAG.json 2
fi
if [ "${EXTRA:-1}" = 1 ]; then
  # action-level workloads: C4 transfers through the typed batch and as raw TokenRequests, C5 mixed
  step bench_transfer 300 python3 -u bench.py --workload transfer --steps 96 --warmup 4
  step bench_request 300 python3 -u bench.py --workload request --steps 96 --warmup 4
  step bench_mixed 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4
  step bench_audit 200 python3 -u bench.py --workload audit --steps 64 --warmup 4
  step bench_prove 300 python3 -u bench.py --workload prove --batch 16384 --steps 12 --warmup 2
  for w in transfer request mixed audit prove; do grep '^{' $OUT/bench_$w.log | tail -1 > $OUT/bench_$w.json; done
fi
echo "== done"
