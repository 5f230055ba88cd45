export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_idemix.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/idemix_pt.log 2>&1; rc=$?; tail -15 gpurun_out/idemix_pt.log; [ $rc -eq 0 ] || exit 1
bash tools/s20_sweep.sh
