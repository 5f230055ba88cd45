set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_headline.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
L=fabric-token-sdk_amd/lib/libfts_gpu.so
TAG=r05v LIBS="fabric-token-sdk_amd/lib/ab/head.so $L $L@FTS_WORK_BS=256" bash tools/ab_session.sh burst s512 burst || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 tools/burst.py --steps 20 --reps 3 > $O/burst.log 2>&1 || { tail -20 $O/burst.log; exit 1; }
python3 tools/trace_burst.py $(find $O/tr -name "*kernel_trace.csv" | head -1) > $O/burst_trace.txt
tail -1 $O/burst_trace.txt
