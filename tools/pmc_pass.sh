#!/bin/bash
# PMC counters of isolated 81,920-proof passes (tools/pass_times.py), one
# rocprofv3 --pmc run per counter group (gpurun rules: <= 8 SQ_, 4 TCC_ per run),
# for each LIBS entry (path[@K=V,...]) -> $OUT/pmc_<arm>.txt / .json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
GROUPS_=${PMC_GROUPS:-"SQ_INSTS_VALU,SQ_INSTS_VALU_INT64,SQ_INSTS_SALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_LDS FETCH_SIZE WRITE_SIZE"}
for spec in ${LIBS:-fabric-token-sdk_amd/lib/libfts_gpu.so}; do
  L=${spec%%@*}; E=""; [[ $spec == *@* ]] && E=${spec#*@}
  n=$(basename $L .so)${E:+_${E//[=,]/_}}
  dirs=""
  i=0
  for g in $GROUPS_; do
    i=$((i + 1))
    d=$OUT/pmc_${n}_$i
    rm -rf $d
    ( [ -n "$E" ] && export $(echo $E | tr ',' ' '); export FTS_LIB=$L
      timeout -s KILL 120 rocprofv3 --pmc $(echo $g | tr ',' ' ') -f csv -d $d -o run -- python3 tools/pass_times.py 81920 > $d.log 2>&1 ) || { echo "pmc $n $g FAILED"; tail -20 $d.log; exit 1; }
    dirs="$dirs $d"
  done
  python3 tools/pmc_sum.py $dirs --json $OUT/pmc_$n.json > $OUT/pmc_$n.txt
  echo "== $n"; cat $OUT/pmc_$n.txt
done
