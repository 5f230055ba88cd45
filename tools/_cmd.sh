set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p2; mkdir -p $O
L=fabric-token-sdk_amd/lib/libfts_gpu.so
TAG=r05p2 LIBS="$L $L@FTS_WAVE_PRIO=022223313133 $L@FTS_WAVE_PRIO=022333313133" bash tools/trace_iso.sh > $O/traces.txt 2>&1 || exit 1
grep "^==\|pass span" $O/traces.txt
TAG=r05p2 LIBS="$L $L@FTS_WAVE_PRIO=022223313133 $L@FTS_WAVE_PRIO=022333313133" bash tools/ab_session.sh burst s512
