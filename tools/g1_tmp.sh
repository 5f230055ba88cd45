set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b; mkdir -p $O
T="timeout -k 10"
for lib in fabric-token-sdk_amd/lib/libfts_gpu.so fabric-token-sdk_amd/lib/ab/prio3.so; do
  for sp in 0 20480; do
    FTS_LIB=$lib FTS_SUBPASS=$sp $T 200 python3 -u tools/burst.py --steps 20 --reps 9 --tag $(basename $lib)-sp$sp >> $O/burst.log 2>&1 || exit 1
  done
  FTS_LIB=$lib $T 200 python3 -u tools/pass_times.py 4096 81920 >> $O/pass.log 2>&1 || exit 1
done
echo bursts done
$T 900 python3 -u -m pytest tests/test_gpu_c5.py tests/test_gpu_knobs.py tests/test_gpu_msm.py tests/test_idemix_identity.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest rc=$?
