#!/bin/bash
# Round-2 measurement session (run from the repo root on the gpurun box):
#   smoke -> [pytest -m gpu] -> bench (driver shape, then long) -> rocprofv3
#   kernel-trace stats -> PMC passes (FETCH_SIZE, WRITE_SIZE, VALU; one group per
#   run) + FETCH_SIZE calibration -> traffic JSON -> action-level workloads.
# Every GPU step has its own time limit; the first failure ends the script.
# Env: TESTS=1 (run pytest -m gpu), PMC=0 (skip counters), EXTRA=0 (skip workloads),
#      BENCH=0 (skip the two headline benches), TAG (output subdirectory).
set -o pipefail
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -30 $OUT/$name.log; exit 1; fi
}
json() { grep '^{' $OUT/$1.log | tail -1 > $OUT/$1.json; }
step smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()"
if [ "${TESTS:-0}" = 1 ]; then
  step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  tail -3 $OUT/pytest_gpu.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench_s20 300 python3 -u bench.py --steps 20 --warmup 5
  json bench_s20
  step bench 600 python3 -u bench.py --steps 512 --warmup 64
  json bench
  cut -c1-600 $OUT/bench.json
fi
if [ "${PROF:-1}" = 1 ]; then
  rm -rf $OUT/prof
  step rocprof 400 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof -o run -- python3 bench.py --steps 256 --warmup 64 --roofline-steps 6 --cpu-sample 0
  json rocprof
  python3 tools/prof_summary.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 6 $OUT/prof/isolated.json
fi
if [ "${PMC:-1}" = 1 ]; then
  PB="python3 bench.py --steps 8 --warmup 8 --roofline-steps 2 --cpu-sample 0"
  rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_valu $OUT/pmc_calib
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_fetch -o run -- $PB
  json pmc_fetch
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_write -o run -- $PB
  step pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -T -f csv -d $OUT/pmc_valu -o run -- $PB
  step pmc_calib 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_calib -o run -- fabric-token-sdk_amd/lib/fetch_calib
  json pmc_calib
  python3 tools/pmc_r02.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_calib $OUT/pmc_calib.json $OUT/pmc_fetch.json 2 $OUT/traffic_$TAG.json $OUT/pmc_valu
fi
if [ "${EXTRA:-1}" = 1 ]; then
  step bench_transfer 300 python3 -u bench.py --workload transfer --steps 96 --warmup 4
  step bench_mixed 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4
  step bench_request 300 python3 -u bench.py --workload request --steps 96 --warmup 4
  step bench_msm 300 python3 -u bench.py --workload msm --msm-log 20 --steps 32 --warmup 4
  step bench_msm22 300 python3 -u bench.py --workload msm --msm-log 22 --steps 16 --warmup 2
  step bench_audit 200 python3 -u bench.py --workload audit --steps 64 --warmup 4
  step bench_prove 300 python3 -u bench.py --workload prove --batch 16384 --steps 12 --warmup 2
  step bench_ecdsa 300 python3 -u bench.py --workload ecdsa --steps 64 --warmup 4
  step bench_idemix 300 python3 -u bench.py --workload idemix --steps 32 --warmup 4
  step bench_idemix_fbn 300 python3 -u bench.py --workload idemix --idemix-curve fp256bn --steps 32 --warmup 4
  for w in transfer mixed request msm msm22 audit prove ecdsa idemix idemix_fbn; do json bench_$w; done
fi
echo "== done $(date +%T)"
