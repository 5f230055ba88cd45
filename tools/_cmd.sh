set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05mc; mkdir -p $O
L=fabric-token-sdk_amd/lib/libfts_gpu.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
TAG=r05mc LIBS="$L $L@FTS_MSM_MAXC=15 $L@FTS_MSM_MAXC=14" bash tools/trace_iso.sh > $O/traces.txt 2>&1 || exit 1
grep "^==\|pass span" $O/traces.txt
TAG=r05mc LIBS="$L $L@FTS_MSM_MAXC=15 $L@FTS_MSM_MAXC=14" bash tools/ab_session.sh burst s512
