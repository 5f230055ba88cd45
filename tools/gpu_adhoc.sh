# ad-hoc GPU step of the current change: fallback tests + C5 line + burst timeline of the 20-step headline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_rp.py tests/test_gpu_headline.py tests/test_gpu_actions.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4 --cpu-sample 0 > $O/bench_mixed.log 2>&1 || { tail $O/bench_mixed.log; exit 1; }
grep '^{' $O/bench_mixed.log | tail -1 > $O/bench_mixed.json
python3 -c "import json; d=json.load(open('$O/bench_mixed.json')); print('mixed', d['value'], d['isolated_call_ms'], d['fallback'], d['fallback_pipelined'])"
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 tools/burst.py --steps 20 --reps 3 > $O/burst.log 2>&1 || { tail $O/burst.log; exit 1; }
tail -3 $O/burst.log
python3 tools/burst_timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 150 > $O/burst_timeline.txt
head -150 $O/burst_timeline.txt
