#!/bin/bash
# The measurement recipe behind profiles/ (run on the gpurun box from the repo root):
#   bash tools/gpu_session.sh STEP...     STEP in: smoke tests rp prof pmc tamper identity identity_pmc msm_pmc extra
# smoke     __graft_entry__.smoke()
# tests     pytest -m gpu (full suite)
# rp        C2 headline, driver shape (20 steps) and steady state (512 steps)
# s20x5     five consecutive driver-shape runs (20 steps, no CPU columns)
# prof      rocprofv3 --kernel-trace --stats of the headline; isolated roofline pass summary
# pmc       FETCH_SIZE / WRITE_SIZE / SQ_* passes (one counter group per run) + FETCH_SIZE
#           calibration -> traffic_$TAG.json (tools/pmc_traffic.py)
# tamper    C2 with 1 % tampered proofs; one bad proof per 81,920-proof pass vs clean (160 steps)
# identity  idemix identity validity, both curves, + rocprofv3 stats
# identity_pmc  FETCH_SIZE / WRITE_SIZE per identity kernel (BN254) -> identity_traffic_$TAG.json
# msm_pmc   FETCH_SIZE / WRITE_SIZE per MSM kernel of C3 at 2^22 points -> msm22_traffic_$TAG.json
# extra     C3-C5 and SURVEY 8f workloads
# Every GPU step has its own time limit; the first failure ends the script.
# Output: gpurun_out/$TAG (TAG default r05).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -30 $OUT/$name.log; exit 1; fi
}
json() { grep '^{' $OUT/$1.log | tail -1 > $OUT/$1.json; cut -c1-400 $OUT/$1.json; }
for s in "$@"; do case $s in
  smoke) step smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
  tests) step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
         tail -2 $OUT/pytest_gpu.log ;;
  s20x5) for i in 1 2 3 4 5; do  # the driver-shape line, five consecutive runs
           step bench_s20_$i 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --host-steps 0
           json bench_s20_$i
         done ;;
  rp) step bench_s20 300 python3 -u bench.py --steps 20 --warmup 5; json bench_s20
      step bench 600 python3 -u bench.py --steps 512 --warmup 64; json bench ;;
  prof) rm -rf $OUT/prof
        step rocprof 400 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof -o run -- python3 bench.py --steps 256 --warmup 64 --roofline-steps 6 --cpu-sample 0 --host-steps 0
        json rocprof
        python3 tools/prof_summary.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 6 $OUT/prof/isolated.json ;;
  pmc) PB="python3 bench.py --steps 8 --warmup 8 --roofline-steps 2 --cpu-sample 0 --host-steps 0"
       rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_valu $OUT/pmc_calib
       step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_fetch -o run -- $PB
       json pmc_fetch
       step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_write -o run -- $PB
       step pmc_valu 300 rocprofv3 --pmc VALUBusy SIMD_UTILIZATION SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_SALU -T -f csv -d $OUT/pmc_valu -o run -- $PB
       step pmc_calib 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_calib -o run -- fabric-token-sdk_amd/lib/fetch_calib
       json pmc_calib
       python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_calib $OUT/pmc_calib.json $OUT/pmc_fetch.json 2 $OUT/traffic_$TAG.json $OUT/pmc_valu ;;
  tamper) step bench_tamper 300 python3 -u bench.py --steps 20 --warmup 5 --tamper 0.01; json bench_tamper
          step bench_clean160 300 python3 -u bench.py --steps 160 --warmup 20 --host-steps 0 --cpu-sample 0; json bench_clean160
          step bench_onebad160 300 python3 -u bench.py --steps 160 --warmup 20 --host-steps 0 --cpu-sample 0 --tamper 1e-9 --tamper-every 20
          json bench_onebad160 ;;
  identity_pmc) IB="python3 bench.py --workload identity --idemix-curve bn254 --steps 2 --warmup 1 --cpu-sample 0 --action-inflight 1"
          rm -rf $OUT/pmc_id_fetch $OUT/pmc_id_write
          step pmc_id_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_id_fetch -o run -- $IB
          step pmc_id_write 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_id_write -o run -- $IB
          python3 tools/pmc_kernels.py $OUT/pmc_id_fetch $OUT/pmc_id_write $OUT/identity_traffic_$TAG.json k_idv ;;
  msm_pmc) MB="python3 bench.py --workload msm --msm-log 22 --steps 2 --warmup 1 --cpu-sample 0"
          rm -rf $OUT/pmc_msm_fetch $OUT/pmc_msm_write
          step pmc_msm_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/pmc_msm_fetch -o run -- $MB
          json pmc_msm_fetch
          step pmc_msm_write 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/pmc_msm_write -o run -- $MB
          python3 tools/pmc_kernels.py $OUT/pmc_msm_fetch $OUT/pmc_msm_write $OUT/msm22_traffic_$TAG.json k_msm k_rs ;;
  identity) for c in bn254 fp256bn; do
              step bench_identity_$c 300 python3 -u bench.py --workload identity --idemix-curve $c --steps 40 --warmup 4; json bench_identity_$c
            done
            rm -rf $OUT/prof_identity
            step prof_identity 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof_identity -o prof -- python3 bench.py --workload identity --steps 4 --warmup 1 --cpu-sample 0 ;;
  extra) step bench_transfer 300 python3 -u bench.py --workload transfer --steps 96 --warmup 4
         step bench_mixed 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4
         step bench_request 300 python3 -u bench.py --workload request --steps 96 --warmup 4
         step bench_msm22 300 python3 -u bench.py --workload msm --msm-log 22 --steps 16 --warmup 2
         step bench_audit 200 python3 -u bench.py --workload audit --steps 64 --warmup 4
         step bench_prove 300 python3 -u bench.py --workload prove --batch 16384 --steps 12 --warmup 2
         step bench_ecdsa 300 python3 -u bench.py --workload ecdsa --steps 64 --warmup 4
         step bench_idemix 300 python3 -u bench.py --workload idemix --steps 32 --warmup 4
         for w in transfer mixed request msm22 audit prove ecdsa idemix; do json bench_$w; done ;;
  *) echo "unknown step $s"; exit 2 ;;
esac; done
echo "== done $(date +%T)"
