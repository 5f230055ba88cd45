set -o pipefail
mkdir -p gpurun_out/x0ab
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py -k "x0_split" > gpurun_out/x0ab/t.log 2>&1 || exit 1
for i in 1 2; do
  for v in 1 3; do
    FTS_X0_SPLIT=$v timeout -k 10 200 python bench.py --inflight 1 --steps 30 --warmup 5 --cpu-sample 0 --distinct 8 > gpurun_out/x0ab/lone_${v}_$i.json 2> gpurun_out/x0ab/lone_${v}_$i.err || exit 1
  done
done
for v in 1 3; do
  FTS_X0_SPLIT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/x0ab/s20_${v}.json 2> gpurun_out/x0ab/s20_${v}.err || exit 1
done
