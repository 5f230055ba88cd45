set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e; mkdir -p $O
T="timeout -k 10"
$T 600 python3 -u -m pytest tests/test_idemix_identity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_id.log 2>&1 || exit 1
$T 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_s20.log 2>&1
echo rc=$?
