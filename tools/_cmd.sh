set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h; mkdir -p $O
FTS_RLC_FORK=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
TAG=r05h LIBS="fabric-token-sdk_amd/lib/libfts_gpu.so@FTS_RLC_FORK=4" bash tools/trace_iso.sh
rm -rf $O/bt
FTS_RLC_FORK=4 FTS_GATHER_TARGET=81920 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/bt -o run -- python3 tools/burst.py --steps 20 --reps 2 > $O/bt.log 2>&1 || { tail $O/bt.log; exit 1; }
python3 tools/burst_timeline.py $(find $O/bt -name "*kernel_trace.csv" | head -1) 150 > $O/bt.txt; cat $O/bt.txt | head -80
TAG=r05h LIBS="fabric-token-sdk_amd/lib/libfts_gpu.so@FTS_GATHER_TARGET=81920 fabric-token-sdk_amd/lib/libfts_gpu.so@FTS_RLC_FORK=4,FTS_GATHER_TARGET=81920 fabric-token-sdk_amd/lib/libfts_gpu.so@FTS_RLC_FORK=4" bash tools/ab_session.sh burst s512 s20
