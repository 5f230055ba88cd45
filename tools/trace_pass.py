"""Timeline of the LAST range-proof pass in a rocprofv3 kernel trace: every
kernel of that pass with its start / end (us, relative to the pass's first
kernel) and duration, so the critical path of one isolated pass is visible.
  python tools/trace_pass.py <kernel_trace.csv> [first_kernel=k_rp_decode]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_rp_decode"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("fts::", ""),
             int(r["Grid_Size_X"]), r.get("Queue_Id", "")) for r in rows)
starts = [i for i, e in enumerate(ev) if e[2].startswith(first)]
ev = ev[starts[-1]:]
t0 = ev[0][0]
end = max(e[1] for e in ev)
print("pass span %.1f us" % ((end - t0) / 1e3))
for s, e, name, grid, q in ev:
    print("%8.1f %8.1f %7.1f  %-22s grid=%-8d q=%s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, name[:22], grid, q))
