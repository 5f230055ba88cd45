# ad-hoc GPU step: identity pairing memory traffic (PMC) and in-flight scaling
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i; mkdir -p $O; rm -rf $O/pf $O/pw
B="python3 bench.py --workload identity --steps 2 --warmup 1 --cpu-sample 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $O/pf -o run -- $B > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $O/pw -o run -- $B > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("pf", "pw"):
    f = glob.glob("gpurun_out/r03i/%s/**/*counter_collection.csv" % tag, recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0][-30:], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        if "idv" in k: print(tag, k, c, "per dispatch avg %.3e" % (sum(v) / len(v)), "n", len(v))
PY
for f in 1 3 6; do
  timeout -k 10 200 python3 bench.py --workload identity --steps 12 --warmup 2 --cpu-sample 0 --action-inflight $f > $O/if$f.log 2>&1 || { tail $O/if$f.log; exit 1; }
  grep '^{' $O/if$f.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('inflight $f', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
