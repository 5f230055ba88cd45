set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_rp.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
L=fabric-token-sdk_amd/lib/libfts_gpu.so
TAG=r05w LIBS="fabric-token-sdk_amd/lib/ab/prelat.so $L" bash tools/ab_session.sh s512 || exit 1
TAG=r05w LIBS="$L $L@FTS_GT1=1024,FTS_GT2_MIN=256 $L@FTS_GT1=1024 $L@FTS_GT1=2048,FTS_GT2_MIN=256" bash tools/ab_session.sh onebad
