set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05sp2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_rp.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 python3 -u bench.py --workload msm --msm-log 22 --steps 16 --warmup 2 > $O/bench_msm22.log 2>&1 || { tail -20 $O/bench_msm22.log; exit 1; }
grep '^{' $O/bench_msm22.log | tail -1 > $O/bench_msm22.json
python3 -c "import json; d=json.load(open('$O/bench_msm22.json')); print(d['value'], d['kernel_ms'], d['cpu_baseline']['value'])"
