#!/bin/bash
# A/B of library builds on one gpurun box (the round's main measurement loop):
#   TAG=r05a LIBS="fabric-token-sdk_amd/lib/ab/base.so fabric-token-sdk_amd/lib/libfts_gpu.so@FTS_X=0,FTS_Y=1" \
#     bash tools/ab_session.sh [smoke] [tests] [burst] [pass] [s512]
# (a LIBS entry is a library path, optionally @ comma-separated environment settings)
# tests  pytest -m gpu with the in-tree library (the candidate)
# burst  tools/burst.py medians of 9 driver-shaped 20-batch bursts, libraries alternating (2 rounds)
# pass   tools/pass_times.py: per-kernel HIP-event spans of one isolated 81,920-proof pass, per library
# s512   bench.py --steps 512 per library (steady state)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
LIBS=${LIBS:-fabric-token-sdk_amd/lib/libfts_gpu.so}
# run "$@" with the library and environment of spec $1 (path[@K=V,...]); arm name in $ARM
arm() {
  local spec=$1; shift
  local L=${spec%%@*} E=""
  [[ $spec == *@* ]] && E=${spec#*@}
  ARM=$(basename $L .so)${E:+_${E//[=,]/_}}
  ( [ -n "$E" ] && export $(echo $E | tr ',' ' '); export FTS_LIB=$L; "$@" ) || exit 1
}
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -30 $OUT/$name.log; exit 1; fi
}
for s in "$@"; do case $s in
  smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"; tail -1 $OUT/smoke.log ;;
  tests) step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
         tail -2 $OUT/pytest_gpu.log ;;
  burst) for r in 1 2; do for L in $LIBS; do
           arm $L true; n=$ARM
           arm $L step burst_${n}_$r 240 python3 -u tools/burst.py --steps 20 --reps 9 --tag $n
           grep -i median $OUT/burst_${n}_$r.log | tail -1
         done; done ;;
  pass) for L in $LIBS; do
          arm $L true; n=$ARM
          arm $L step pass_$n 240 python3 -u tools/pass_times.py 81920 81920
          tail -2 $OUT/pass_$n.log
        done ;;
  s512) for L in $LIBS; do
          arm $L true; n=$ARM
          arm $L step s512_$n 400 python3 -u bench.py --steps 512 --warmup 64 --cpu-sample 0 --host-steps 0
          grep '^{' $OUT/s512_$n.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$n', d['value'], d['ms_per_step'], d['isolated_pass'], d['merged_batches_avg'])"
        done ;;
  s20) for L in $LIBS; do
          arm $L true; n=$ARM
          arm $L step s20_$n 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --host-steps 0
          grep '^{' $OUT/s20_$n.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$n', d['value'], d['ms_per_step'], d['isolated_pass'], d['merged_batches_avg'])"
        done ;;
  onebad) for L in $LIBS; do
          arm $L true; n=$ARM
          arm $L step onebad_$n 300 python3 -u bench.py --steps 160 --warmup 20 --host-steps 0 --cpu-sample 0 --tamper 1e-9 --tamper-every 20
          grep '^{' $OUT/onebad_$n.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$n onebad', d['value'], d['ms_per_step'], d['merged_batches_avg'])"
          arm $L step tamper_$n 300 python3 -u bench.py --steps 20 --warmup 5 --host-steps 0 --cpu-sample 0 --tamper 0.01
          grep '^{' $OUT/tamper_$n.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$n tamper1%', d['value'], d['ms_per_step'], d['merged_batches_avg'])"
        done ;;
  *) echo "unknown step $s"; exit 2 ;;
esac; done
echo "== done $(date +%T)"
