"""Per-kernel durations from a rocprofv3 kernel trace of bench.py:
the LAST R dispatches of every kernel are the bench's isolated roofline pass
(one batch alone on the GPU, run after the timed region), so their average is
what bench.py's roofline.kernel_ms must agree with; all dispatches are
summarised too (the pipelined timed region dominates them).

    python tools/prof_summary.py <run_kernel_trace.csv> <R> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict

path, R, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader(open(path)))
by = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("fts::", "")
    by[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                     int(r["Grid_Size_X"])))
out = {}
for name, v in sorted(by.items()):
    v.sort()
    last = v[-R:]
    out[name] = {"calls": len(v), "avg_us_all": round(sum(d for _, d, _ in v) / len(v) / 1e3, 2),
                 "isolated_calls": len(last), "isolated_avg_us": round(sum(d for _, d, _ in last) / len(last) / 1e3, 2),
                 "isolated_grid": last[-1][2]}
json.dump(out, open(dst, "w"), indent=1)
for k in ("k_rp_fixed_exact", "k_rp_com_var", "k_msm_chunks", "k_rp_x0_hash"):
    if k in out:
        print(k, out[k])
