# ad-hoc GPU step of the current change: group-test + latency A/B (see tools/README.md)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_rp.py tests/test_gpu_headline.py tests/test_gpu_actions.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 100 python3 tools/pass_times.py 4096 > $O/pass4k.log 2>&1 && cat $O/pass4k.log || exit 1
rm -rf $O/trace
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 tools/pass_times.py 4096 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python3 tools/trace_pass.py $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/lone_timeline.txt
head -45 $O/lone_timeline.txt
timeout -k 10 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4 --cpu-sample 0 > $O/bench_mixed.log 2>&1 || { tail $O/bench_mixed.log; exit 1; }
grep '^{' $O/bench_mixed.log | tail -1 > $O/bench_mixed.json
python3 -c "import json; d=json.load(open('$O/bench_mixed.json')); print('mixed', d['value'], d['fallback'])"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --tamper 0.01 --cpu-sample 0 > $O/bench_tamper.log 2>&1 || { tail $O/bench_tamper.log; exit 1; }
grep '^{' $O/bench_tamper.log | tail -1 > $O/bench_tamper.json
python3 -c "import json; d=json.load(open('$O/bench_tamper.json')); print('tamper', d['value'], d['fallback'], d['isolated_batch']['ms'], {k:v for k,v in d['kernel_ms_isolated'].items() if k.startswith('fb:')})"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_s20.log 2>&1 || { tail $O/bench_s20.log; exit 1; }
grep '^{' $O/bench_s20.log | tail -1 > $O/bench_s20.json
python3 -c "import json; d=json.load(open('$O/bench_s20.json')); print('s20', d['value'], d['isolated_batch']['ms'], d['isolated_pass'])"
