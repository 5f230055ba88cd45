set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_headline.py tests/test_gpu_actions.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
TAG=fixed timeout -k 10 200 python3 tools/pass_times.py 4096 8192 16384 32768 || exit 1
rm -rf gpurun_out/tr4k
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/tr4k -o run -- python3 tools/pass_times.py 4096 > gpurun_out/tr4k.log 2>&1 || exit 1
python3 tools/trace_pass.py $(find gpurun_out/tr4k -name "*kernel_trace.csv" | head -1)
