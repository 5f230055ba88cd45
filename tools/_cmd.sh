set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_rp.py tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
PB="python3 bench.py --steps 8 --warmup 8 --roofline-steps 2 --cpu-sample 0 --host-steps 0"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $O/pmc_write -o run -- $PB > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
python3 - <<'PY'
import sys; sys.path.insert(0,'tools')
from pmc_traffic import per_kernel
w=per_kernel('gpurun_out/r05t/pmc_write','WRITE_SIZE')
for k in ('k_msm_split','k_rs_hist','k_rs_pscan','k_rs_scatter','k_rs_part'):
    v=w.get(k,[])[-2:]
    print(k, round(sum(v)/max(1,len(v))*1024/1e6,1),'MB')
PY
L=fabric-token-sdk_amd/lib/libfts_gpu.so
TAG=r05t LIBS="fabric-token-sdk_amd/lib/ab/r05base.so $L fabric-token-sdk_amd/lib/ab/psh6.so" bash tools/ab_session.sh burst s512
TAG=r05t LIBS="fabric-token-sdk_amd/lib/ab/r05base.so $L" bash tools/trace_iso.sh > $O/iso.txt 2>&1; grep "==\|span" $O/iso.txt
