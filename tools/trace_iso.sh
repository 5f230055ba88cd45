#!/bin/bash
# rocprofv3 kernel trace of isolated 81,920-proof passes (tools/pass_times.py) for
# each LIBS entry (path[@K=V,...]); the last pass's timeline -> $OUT/trace_<arm>.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
TAG=${TAG:-trace}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in ${LIBS:-fabric-token-sdk_amd/lib/libfts_gpu.so}; do
  L=${spec%%@*}; E=""; [[ $spec == *@* ]] && E=${spec#*@}
  n=$(basename $L .so)${E:+_${E//[=,]/_}}
  rm -rf $OUT/tr_$n
  ( [ -n "$E" ] && export $(echo $E | tr ',' ' '); export FTS_LIB=$L
    timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/tr_$n -o run -- python3 tools/pass_times.py 81920 > $OUT/tr_$n.log 2>&1 ) || { echo "trace $n FAILED"; tail -20 $OUT/tr_$n.log; exit 1; }
  python3 tools/trace_last_pass.py $(find $OUT/tr_$n -name "*kernel_trace.csv" | head -1) > $OUT/trace_$n.txt
  echo "== $n"; cat $OUT/trace_$n.txt
done
