set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 200 python3 -u tools/burst.py --steps 20 --reps 7 > $O/burst.log 2>&1 &&
timeout -k 10 200 python3 -u tools/pass_times.py 4096 81920 > $O/pass.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 tools/burst.py --steps 20 --reps 3 > $O/trace.log 2>&1 &&
python3 tools/burst_timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 150 > $O/timeline.txt
echo rc=$?
FTS_COM_FIXED_MAX=0 timeout -k 10 300 python3 -u tools/pass_times.py 4096 8192 16384 32768 81920 > gpurun_out/r04a/pass_work.log 2>&1
echo rc2=$?
