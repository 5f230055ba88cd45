"""Timeline of the last range-proof pass in a rocprofv3 kernel trace (the pass
whose k_rp_fixed_exact / k_rp_fixed_all launch is last), relative to its first
kernel: start, end, span, queue, kernel, grid.
    python tools/trace_last_pass.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("fts::", "").replace("void ", "").split("<")[0], r["Queue_Id"],
             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) for r in rows)
fx = [e for e in ev if e[2] in ("k_rp_fixed_exact", "k_rp_fixed_all")]
t_fx = fx[-1][0]
# the pass starts at its k_rp_decode before that launch
dec = [e for e in ev if e[2] == "k_rp_decode" and e[0] <= t_fx]
T0 = dec[-1][0] if dec else t_fx
end = max(e[1] for e in ev)
for s, e, n, q, g in ev:
    if s >= T0:
        print("%8.3f %8.3f %6.3f q%-3s %-28s %d" % ((s - T0) / 1e6, (e - T0) / 1e6, (e - s) / 1e6, q, n, g))
print("pass span %.3f ms" % ((end - T0) / 1e6))
