"""Timeline of the last burst in a rocprofv3 kernel trace of tools/burst.py
(bursts are separated by > 3 ms with no kernel running): per kernel start, end,
span, queue, grid relative to the burst's first kernel, then the burst's kernel
span and the busy fraction (union of kernel intervals).
    python tools/trace_burst.py run_kernel_trace.csv [gap_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
gap = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 3e6
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("fts::", "").replace("void ", "").split("<")[0], r["Queue_Id"],
             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) for r in rows)
bursts, cur, hi = [], [], 0
for e in ev:
    if cur and e[0] > hi + gap:
        bursts.append(cur)
        cur = []
    cur.append(e)
    hi = max(hi, e[1]) if cur[:-1] else e[1]
bursts.append(cur)
b = bursts[-1]
T0 = b[0][0]
for s, e, n, q, g in b:
    print("%8.3f %8.3f %6.3f q%-3s %-28s %d" % ((s - T0) / 1e6, (e - T0) / 1e6, (e - s) / 1e6, q, n, g))
busy, end = 0, T0
for s, e, *_ in b:
    if e > end:
        busy += e - max(s, end)
        end = e
print("bursts %d; last: span %.3f ms, busy %.3f ms" % (len(bursts), (end - T0) / 1e6, busy / 1e6))
