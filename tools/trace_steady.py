"""Steady-state overlap of a rocprofv3 kernel trace of bench.py (512 steps): over
the timed region (the span of the k_rp_fixed_exact launches but the last R
isolated ones), how much of the time each pass-phase runs beside another pass's
work, and the union busy fraction.
    python tools/trace_steady.py run_kernel_trace.csv [R]
Prints: passes, mean fixed-base launch span, the fraction of fixed-base time that
overlaps another pass's chain kernels (hsum/join/com_var/normalize/x0 hash), the
fraction of chain time that overlaps a fixed-base launch, and the busy fraction."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("fts::", "").replace("void ", "").split("<")[0]) for r in rows)
fx = [e for e in ev if e[2] == "k_rp_fixed_exact"]
fx = fx[:-R] if len(fx) > R else fx
T0, T1 = fx[len(fx) // 8][0], fx[-1][1]  # skip the warmup's first passes
CHAIN = {"k_rp_hsum_chunks", "k_rp_hsum_join", "k_rp_com_var", "k_rp_normalize", "k_rp_x0_hash"}
ch = [e for e in ev if e[2] in CHAIN and T0 <= e[0] < T1]
fxs = [e for e in fx if T0 <= e[0] < T1]


def overlap(a, bs):
    s, e = a[0], a[1]
    iv = sorted((max(s, b[0]), min(e, b[1])) for b in bs if b[0] < e and b[1] > s)
    tot, cur = 0, s
    for x, y in iv:
        if y > cur:
            tot += y - max(x, cur)
            cur = y
    return tot


fx_ov = sum(overlap(a, ch) for a in fxs) / max(1, sum(a[1] - a[0] for a in fxs))
ch_ov = sum(overlap(a, fxs) for a in ch) / max(1, sum(a[1] - a[0] for a in ch))
allk = [e for e in ev if T0 <= e[0] < T1]
busy = overlap((T0, T1), allk) / (T1 - T0)
print("passes %d in %.1f ms (%.3f ms per pass); fixed-base span %.3f ms mean" %
      (len(fxs), (T1 - T0) / 1e6, (T1 - T0) / 1e6 / max(1, len(fxs)),
       sum(a[1] - a[0] for a in fxs) / 1e6 / max(1, len(fxs))))
print("fixed-base time beside a chain kernel: %.3f; chain time beside a fixed-base launch: %.3f; busy %.4f"
      % (fx_ov, ch_ov, busy))
