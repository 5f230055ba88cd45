export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "2 16384" "4 4096"; do set -- $cfg
  rm -rf gpurun_out/tr_$1_$2
  FTS_COALESCE_MAX=$2 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/tr_$1_$2 -o run -- python3 bench.py --steps 64 --warmup 16 --lanes $1 --inflight 16 --distinct 1 --cpu-sample 0 --roofline-steps 1 > gpurun_out/tr_$1_$2.log 2>&1 || exit 1
  grep '^{' gpurun_out/tr_$1_$2.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$cfg', round(d['value']), d['merged_batches_avg'])"
done
