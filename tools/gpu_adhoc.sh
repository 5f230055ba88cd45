# ad-hoc GPU step: per-plan MSM chunk size (tests, MSM 2^22, lone batch, headline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_rp.py tests/test_gpu_scale.py tests/test_gpu_headline.py tests/test_gpu_actions.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -40 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 python3 -u bench.py --workload msm --msm-log 22 --steps 16 --warmup 2 --cpu-sample 0 > $O/msm22.log 2>&1 || { tail $O/msm22.log; exit 1; }
grep '^{' $O/msm22.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('msm22', d['value'], d['ms_per_step'], d['kernel_ms'])"
timeout -k 10 100 python3 tools/pass_times.py 4096 81920 > $O/pass.log 2>&1 && cat $O/pass.log | cut -c1-600 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/s20.log 2>&1 || { tail $O/s20.log; exit 1; }
grep '^{' $O/s20.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('s20', d['value'], d['isolated_batch']['ms'], d['isolated_pass']['ms'])"
timeout -k 10 300 python3 -u bench.py --steps 512 --warmup 64 --cpu-sample 0 > $O/s512.log 2>&1 || { tail $O/s512.log; exit 1; }
grep '^{' $O/s512.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('s512', d['value'])"
