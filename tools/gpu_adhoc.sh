# ad-hoc GPU step: split-com A/B (FTS_COM_SPLIT) on the isolated 81,920-proof pass, bursts and steady state
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f; mkdir -p $O
FTS_COM_SPLIT=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for sp in 0 1 0 1; do
  FTS_COM_SPLIT=$sp timeout -k 10 120 python3 tools/pass_times.py 81920 > $O/pass.log 2>&1 || { tail $O/pass.log; exit 1; }
  echo "split=$sp: $(cat $O/pass.log | tr ' ' '\n' | grep -E 'wall|com_|hsum|fixed_exact|k_rp_xd|x0_prefix' | tr '\n' ' ')"
done
bash tools/sweep.sh tools/sweeps/com_split.txt || exit 1
