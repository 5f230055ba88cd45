set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t; mkdir -p $O
T="timeout -k 10"
A=fabric-token-sdk_amd/lib/ab
L=fabric-token-sdk_amd/lib/libfts_gpu.so
$T 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_idemix_identity.py > $O/pytest.log 2>&1 || exit 1
for v in $A/base.so $L $A/base.so $L; do
  FTS_LIB=$v $T 200 python3 -u bench.py --workload identity --idemix-curve bn254 --steps 40 --warmup 4 --cpu-sample 0 >> $O/id_ab.txt 2>> $O/id_ab.err || exit 1
done
echo rc=$?
