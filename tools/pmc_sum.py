"""Per-kernel averages per dispatch of every counter in one or more rocprofv3
--pmc output directories (tools/pmc_pass.sh), as a table:
    python tools/pmc_sum.py <dir> [<dir> ...] [--json out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if out_json in args:
    args.remove(out_json)
vals = defaultdict(lambda: defaultdict(list))
for d in args:
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0].replace("fts::", "").replace("void ", "").split("<")[0]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in vals for c in vals[k]})
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
print("%-26s %s" % ("kernel", " ".join("%14s" % c[-14:] for c in names)))
for k in sorted(res, key=lambda k: -res[k].get(names[0], 0)):
    print("%-26s %s" % (k[:26], " ".join("%14.4g" % res[k].get(c, float("nan")) for c in names)))
if out_json:
    json.dump(res, open(out_json, "w"), indent=1, sort_keys=True)
