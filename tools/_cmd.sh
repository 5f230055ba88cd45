set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 200 --timeout-method thread -k "locator" > $O/pt0.log 2>&1 || { tail -40 $O/pt0.log; exit 1; }
tail -1 $O/pt0.log
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_rp.py tests/test_gpu_c5.py tests/test_gpu_knobs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
L=fabric-token-sdk_amd/lib/libfts_gpu.so
TAG=r05y LIBS="fabric-token-sdk_amd/lib/ab/preloc.so $L" bash tools/ab_session.sh onebad onebad
