"""Where the device time of a steady state goes: from a rocprofv3 kernel trace,
over the window [first launch of KERNEL + skip, last launch of KERNEL], the sum of
each kernel's durations (ms per call of the workload when --calls is given), its
share of that sum, and the union busy fraction of the window.
    python tools/trace_busy.py run_kernel_trace.csv [--anchor k_rp_fixed_exact] [--skip 0.15] [--calls N]
Kernel durations overlap (several lanes / streams), so the sums are device time,
not wall time; the union busy fraction says whether the GPU ever idles."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="k_rp_fixed_exact")
    ap.add_argument("--skip", type=float, default=0.15, help="fraction of the anchor launches skipped (warmup)")
    ap.add_argument("--drop-last", type=int, default=0, help="anchor launches dropped at the end (isolated runs)")
    ap.add_argument("--calls", type=float, default=0, help="workload calls in the window (per-call ms)")
    a = ap.parse_args()
    ev = []
    for r in csv.DictReader(open(a.trace)):
        nm = r["Kernel_Name"].split("(")[0].replace("fts::", "").replace("void ", "").split("<")[0].strip()
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm))
    ev.sort()
    anc = [e for e in ev if e[2] == a.anchor]
    if a.drop_last:
        anc = anc[:-a.drop_last]
    t0, t1 = anc[int(len(anc) * a.skip)][0], anc[-1][1]
    win = [e for e in ev if t0 <= e[0] < t1]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in win:
        tot[n] += (e - s) / 1e6
        cnt[n] += 1
    busy, cur = 0, t0
    for s, e, _ in win:
        if e > cur:
            busy += e - max(s, cur)
            cur = e
    span = (t1 - t0) / 1e6
    allk = sum(tot.values())
    print("window %.3f ms, %d launches, union busy %.4f, kernel-time sum %.3f ms (%.2fx the window)"
          % (span, len(win), busy / 1e6 / span, allk, allk / span))
    for n, v in sorted(tot.items(), key=lambda x: -x[1]):
        per = (" %.4f ms/call" % (v / a.calls)) if a.calls else ""
        print("  %-28s %9.3f ms %6.2f%% %6d launches%s" % (n, v, 100 * v / allk, cnt[n], per))


if __name__ == "__main__":
    main()
