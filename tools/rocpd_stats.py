"""Per-kernel statistics from a rocprofv3 SQLite output (rocpd `*_results.db`, the
format rocprofv3 writes without `-f csv`): calls, total / average / min / max ms,
share of the kernel time, and the kernel's VGPR / AGPR / SGPR / scratch figures.
    python tools/rocpd_stats.py run_results.db [--csv out.csv]"""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    sym = {r[0]: r[1:] for r in c.execute(
        "select id, display_name, arch_vgpr_count, accum_vgpr_count, sgpr_count, private_segment_size "
        "from rocpd_info_kernel_symbol")}
    d = collections.defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        d[kid].append((e - s) / 1e6)
    tot = sum(sum(v) for v in d.values())
    rows = []
    for kid, v in sorted(d.items(), key=lambda x: -sum(x[1])):
        nm, vg, ag, sg, scr = sym[kid]
        nm = nm.split("(")[0].replace("void ", "")
        rows.append({"kernel": nm, "calls": len(v), "total_ms": round(sum(v), 4), "avg_ms": round(sum(v) / len(v), 4),
                     "min_ms": round(min(v), 4), "max_ms": round(max(v), 4), "pct": round(100 * sum(v) / tot, 2),
                     "vgpr": vg, "agpr": ag, "sgpr": sg, "scratch": scr})
    for r in rows:
        print("%-44s %5d %10.3f %8.4f %6.2f%%  vgpr %s agpr %s scratch %s" % (
            r["kernel"][:44], r["calls"], r["total_ms"], r["avg_ms"], r["pct"], r["vgpr"], r["agpr"], r["scratch"]))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main()
