"""Timeline of the LAST burst in a rocprofv3 kernel trace of tools/burst.py:
the burst starts after the longest idle gap; prints, per hardware queue, the
kernels longer than --min-us with start / end relative to the burst start.
    python tools/burst_timeline.py <kernel_trace.csv> [min_us]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("fts::", ""),
             r.get("Queue_Id", "")) for r in rows)
# busy intervals -> the start of the last burst = end of the last idle gap longer than 2 ms
t_end = ev[0][1]
start = 0
for i, (s, e, n, q) in enumerate(ev):
    if s - t_end > 2_000_000:
        start = i
    t_end = max(t_end, e)
ev = ev[start:]
t0 = ev[0][0]
span = (max(e for _, e, _, _ in ev) - t0) / 1e3
busy = 0.0
cur_s, cur_e = None, None
for s, e, _, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += (cur_e - cur_s) / 1e3
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += (cur_e - cur_s) / 1e3
print("burst span %.1f us, device busy (any kernel) %.1f us, %d kernels" % (span, busy, len(ev)))
byq = defaultdict(list)
for s, e, n, q in ev:
    byq[q].append((s, e, n))
for q, ks in sorted(byq.items()):
    print("queue %s: %.1f .. %.1f us" % (q, (ks[0][0] - t0) / 1e3, (max(e for _, e, _ in ks) - t0) / 1e3))
    for s, e, n in ks:
        if (e - s) / 1e3 >= min_us:
            print("   %8.1f %8.1f %7.1f  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, n[:26]))
