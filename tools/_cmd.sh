set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 bench.py --steps 512 --warmup 64 --cpu-sample 0 --host-steps 0 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep '^{' $O/b.log | cut -c1-200
python3 tools/trace_steady.py $(find $O/tr -name "*kernel_trace.csv" | head -1) 6 | tee $O/steady.txt
