set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ab; mkdir -p $O
T="timeout -k 10"
$T 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_idemix_identity.py > $O/pytest.log 2>&1 || exit 1
for c in bn254 fp256bn bn254 fp256bn; do
  $T 200 python3 -u bench.py --workload identity --idemix-curve $c --steps 40 --warmup 4 --cpu-sample 0 >> $O/id.txt 2>> $O/id.err || exit 1
done
echo rc=$?
