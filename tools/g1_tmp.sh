set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g; mkdir -p $O
T="timeout -k 10"
$T 600 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_knobs.py tests/test_gpu_c5.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
$T 200 python3 -u tools/pass_times.py 4096 81920 > $O/pass.log 2>&1 || exit 1
$T 200 python3 -u tools/burst.py --steps 20 --reps 9 > $O/burst.log 2>&1 || exit 1
$T 300 python3 -u tools/burst.py --steps 512 --reps 2 >> $O/burst.log 2>&1
echo rc=$?
