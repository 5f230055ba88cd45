# ad-hoc GPU step: full-size exact-intermediate parity vs the CPU batch verifier + C5 with the coop per-proof stage
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_scale.py tests/test_gpu_actions.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -40 $O/pt.log; exit 1; }
grep -E "PASS|FAIL" $O/pt.log | tail -8; tail -1 $O/pt.log
timeout -k 10 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4 --cpu-sample 0 > $O/bench_mixed.log 2>&1 || { tail $O/bench_mixed.log; exit 1; }
grep '^{' $O/bench_mixed.log | tail -1 > $O/bench_mixed.json
python3 -c "import json; d=json.load(open('$O/bench_mixed.json')); print('mixed', d['value'], d['isolated_call_ms'], d['fallback'], d['fallback_pipelined']); print({k:v for k,v in d['kernel_ms_isolated'].items() if k.startswith('fb:')})"
