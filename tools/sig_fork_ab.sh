# A/B of FTS_SIG_FORK (sigma fixed-base products on a second slot stream) on C4 / C5,
# alternating on one box, after the action tests (run from the repo root on the GPU box)
set -o pipefail
O=gpurun_out/sigf
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_actions.py tests/test_gpu_c5.py tests/test_gpu_coalesce.py tests/test_gpu_request.py > $O/t.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    FTS_SIG_FORK=$v timeout -k 10 300 python bench.py --workload transfer --steps 40 --warmup 4 --action-inflight 3 --cpu-sample 0 > $O/tr3_${v}_$i.json 2> $O/tr3_${v}_$i.err || exit 1
    FTS_SIG_FORK=$v timeout -k 10 300 python bench.py --workload transfer --steps 60 --warmup 8 --cpu-sample 0 > $O/tr8_${v}_$i.json 2> $O/tr8_${v}_$i.err || exit 1
    FTS_SIG_FORK=$v timeout -k 10 300 python bench.py --workload mixed --steps 40 --warmup 8 --cpu-sample 0 > $O/mx8_${v}_$i.json 2> $O/mx8_${v}_$i.err || exit 1
  done
done
