set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w; mkdir -p $O
T="timeout -k 10"
A=fabric-token-sdk_amd/lib/ab
L=fabric-token-sdk_amd/lib/libfts_gpu.so
$T 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rp.py tests/test_gpu_knobs.py > $O/pytest.log 2>&1 || exit 1
for v in $A/base.so $L $A/base.so $L; do
  FTS_LIB=$v $T 200 python3 -u tools/pass_times.py 81920 >> $O/pass.log 2>&1 || exit 1
  FTS_LIB=$v $T 200 python3 -u tools/burst.py --steps 20 --reps 9 --tag $(basename $v .so) >> $O/burst.log 2>&1 || exit 1
done
echo rc=$?
