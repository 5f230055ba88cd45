set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rp.py tests/test_gpu_headline.py tests/test_gpu_actions.py tests/test_gpu_scale.py tests/test_gpu_multi.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
TAG=fixed timeout -k 10 200 python3 tools/pass_times.py 4096 8192 16384 || exit 1
rm -rf gpurun_out/tr4k gpurun_out/pmc4k
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/tr4k -o run -- python3 tools/pass_times.py 4096 > gpurun_out/tr4k.log 2>&1 || exit 1
python3 tools/trace_pass.py $(find gpurun_out/tr4k -name "*kernel_trace.csv" | head -1)
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -f csv -d gpurun_out/pmc4k -o run -- python3 tools/pass_times.py 4096 > gpurun_out/pmc4k.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc4k/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("fts::", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(acc):
    if not k.startswith("k_"): continue
    d = acc[k]
    print("%-20s " % k[:20] + " ".join("%s=%.3g" % (c.replace("SQ_", ""), v) for c, v in sorted(d.items())))
PY
