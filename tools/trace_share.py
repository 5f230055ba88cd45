"""Per-kernel share of device time in the steady state of a rocprofv3
kernel trace (middle 60 % of the run's kernels):
  python tools/trace_share.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("fts::", ""))
            for r in rows)
ev = [e for e in ev if not e[2].startswith("kt_")]
ev = ev[len(ev) * 4 // 10:-30]
T0, T1 = ev[0][0], max(e[1] for e in ev)
agg = defaultdict(lambda: [0, 0.0])
for s, e, n in ev:
    agg[n][0] += 1
    agg[n][1] += (e - s) / 1e6
tot = sum(a[1] for a in agg.values())
print("window %.1f ms, sum of kernel time %.1f ms (mean %.2f in flight)" % ((T1 - T0) / 1e6, tot, tot / ((T1 - T0) / 1e6)))
for n, a in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-24s %5d %8.2f ms %5.1f%%  avg %8.1f us" % (n[:24], a[0], a[1], 100 * a[1] / tot, 1e3 * a[1] / a[0]))
