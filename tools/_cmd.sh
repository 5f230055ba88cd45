set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "locator or one_bad" > $O/pt0.log 2>&1 || { tail -40 $O/pt0.log; exit 1; }
tail -1 $O/pt0.log
TAG=r05f2 bash tools/gpu_session.sh smoke tests s20x5 rp tamper || exit 1
timeout -k 10 300 python3 -u bench.py --workload msm --msm-log 22 --steps 16 --warmup 2 > $O/bench_msm22.log 2>&1 || { tail -20 $O/bench_msm22.log; exit 1; }
grep '^{' $O/bench_msm22.log | tail -1 > $O/bench_msm22.json; cut -c1-300 $O/bench_msm22.json
timeout -k 10 300 python3 -u bench.py --workload mixed --transfers 4096 --steps 48 --warmup 4 --cpu-sample 0 > $O/bench_mixed.log 2>&1 || { tail -20 $O/bench_mixed.log; exit 1; }
grep '^{' $O/bench_mixed.log | tail -1 > $O/bench_mixed.json
