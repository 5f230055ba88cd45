#!/bin/bash
# Round-2 GPU check: gpu tests, then the driver's bench line (--steps 20) and a
# steady-state bench (--steps 512).  Every GPU step has its own limit; the first
# failure ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -40 $OUT/$name.log; exit 1; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 700 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
  tail -3 $OUT/pytest_gpu.log
fi
step smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()"
for st in ${STEPS_LIST:-20 512}; do
  step bench_s$st 400 python3 -u bench.py --steps $st --warmup 5 ${BENCH_ARGS:-}
  grep '^{' $OUT/bench_s$st.log | tail -1 > $OUT/bench_s$st.json
  python3 - $OUT/bench_s$st.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("steps", d["steps"], "value", d["value"], "ms/step", d["ms_per_step"], "merged", d.get("merged_batches_avg"),
      "iso_batch_ms", d["isolated_batch"]["ms"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
print("kernels", d.get("kernel_ms_isolated"))
print("cpu", d.get("cpu_baseline"))
PY
done
echo "== done"
