"""Concurrency view of a rocprofv3 kernel trace (run_kernel_trace.csv):
per-kernel busy time, the union of busy time (any kernel running), mean
number of kernels in flight, and idle gaps, over a window of the run.
  python tools/trace_analyze.py <kernel_trace.csv> [skip_first_ms]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]),
       r["Queue_Id"], int(r["VGPR_Count"]), int(r["LDS_Block_Size"]), int(r["Scratch_Size"])) for r in rows]
ev.sort()
t0 = ev[0][0] + skip * 1e6
ev = [e for e in ev if e[0] >= t0 and not e[2].startswith("kt_")]
# keep the busiest segment (segments split at host gaps > 20 ms: proving, setup)
segs, cur_seg, end = [], [], 0
for e in ev:
    if cur_seg and e[0] - end > 20e6:
        segs.append(cur_seg)
        cur_seg = []
    cur_seg.append(e)
    end = max(end, e[1])
segs.append(cur_seg)
ev = max(segs, key=len)
T0, T1 = ev[0][0], max(e[1] for e in ev)
span = (T1 - T0) / 1e6
# union + mean concurrency
pts = sorted([(e[0], 1) for e in ev] + [(e[1], -1) for e in ev])
busy, cur, last, area = 0, 0, T0, 0
gaps = []
for t, d in pts:
    if cur > 0:
        busy += t - last
    elif t - last > 20000:
        gaps.append((t - last) / 1e3)
    area += cur * (t - last)
    cur += d
    last = t
print("window %.2f ms, kernels %d, busy(union) %.2f ms (%.1f%%), mean in flight %.2f, idle gaps>20us: %d totalling %.2f ms"
      % (span, len(ev), busy / 1e6, 100 * busy / (T1 - T0), area / (T1 - T0), len(gaps), sum(gaps) / 1e3))
agg = defaultdict(lambda: [0, 0.0, 0, 0, 0, 0])
for s, e, n, g, q, v, l, sc in ev:
    a = agg[n]
    a[0] += 1
    a[1] += (e - s) / 1e6
    a[2] = max(a[2], g)
    a[3], a[4], a[5] = v, l, sc
print("%-22s %6s %9s %9s %8s %5s %6s %6s" % ("kernel", "calls", "sum_ms", "avg_us", "maxgrid", "vgpr", "lds", "scr"))
for n, a in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-22s %6d %9.2f %9.1f %8d %5d %6d %6d" % (n[:22], a[0], a[1], 1e3 * a[1] / a[0], a[2], a[3], a[4], a[5]))
print("queues:", sorted(set(e[4] for e in ev)))
