set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o tr -- python3 tools/pass_times.py 4096 > gpurun_out/tr.log 2>&1 || { tail -20 gpurun_out/tr.log; exit 1; }
f=$(find gpurun_out/tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_pass.py $f
