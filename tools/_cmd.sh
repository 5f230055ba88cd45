set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05last; mkdir -p $O
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_s20.log 2>&1 || { tail -20 $O/bench_s20.log; exit 1; }
grep '^{' $O/bench_s20.log | tail -1 > $O/bench_s20.json
python3 -c "import json; d=json.load(open('$O/bench_s20.json')); print(d['value'], d['merged_batches_avg'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source'], d['library'].get('matches_build_record'))"
