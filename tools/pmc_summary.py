"""Summarise rocprofv3 --pmc CSVs (one counter group per run, tools/gpu_round.sh)
into per-kernel averages over the bench's dispatches -> profiles/traffic_<tag>.json.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  Per
MI355X_MICROARCH.md (HBM section), FETCH_SIZE reads exactly half the bytes of
wide coalesced streaming reads on gfx950, so ``fetch_bytes_corrected`` =
2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are
memory-side (L2 <-> fabric) traffic and count Infinity-Cache hits.

    python tools/pmc_summary.py gpurun_out r01f profiles/traffic_r01.json [R]

With R, the per-kernel averages of the LAST R dispatches (bench.py's isolated
roofline pass, one batch alone on the GPU) are stored as "<kernel>@isolated".
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path, last=0):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    for row in rows:
        acc[row["Kernel_Name"].split("(")[0].replace("fts::", "")][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if last:
        acc = {k: {c: v[-last:] for c, v in ctrs.items()} for k, ctrs in acc.items()}
    return acc


def main():
    out_dir, tag, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    merged = defaultdict(dict)
    for d in glob.glob(os.path.join(out_dir, "pmc_*_%s" % tag)):
        for csvp in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for suffix, lst in (("", 0), ("@isolated", last)):
                if suffix and not last:
                    continue
                for kern, ctrs in load(csvp, lst).items():
                    for c, vals in ctrs.items():
                        merged[kern + suffix][c] = sum(vals) / len(vals)
                        merged[kern + suffix]["dispatches"] = len(vals)
    res = {}
    for kern, c in sorted(merged.items()):
        r = {k: round(v, 3) for k, v in c.items()}
        if "FETCH_SIZE" in c:
            r["fetch_bytes_corrected"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            r["write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            r["valu_active_per_wave_cycle"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
        res[kern] = r
    with open(dst, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k in ("k_rp_fixed_exact", "k_rp_fixed_exact@isolated", "k_msm_chunks", "k_rp_com_var"):
        if k in res:
            print(k, res[k])


if __name__ == "__main__":
    main()
