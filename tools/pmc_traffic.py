"""HBM traffic per launch for bench.py's `roofline.traffic`, from separate
rocprofv3 PMC passes over the same bench command (tools/gpu_round_r02.sh).

Inputs: the FETCH_SIZE and WRITE_SIZE counter CSVs of the bench command, the
FETCH_SIZE CSV of lib/fetch_calib with the byte counts it printed, the bench
JSON line of the PMC command (for the isolated pass size), and R = its
--roofline-steps.  The LAST R dispatches of every kernel are bench.py's isolated
roofline pass; their average is stored under "<kernel>@pass<proofs>".

FETCH_SIZE counts memory-side read requests (KiB).  Its ratio to the bytes a
kernel really reads depends on the access pattern, so it is calibrated with
kernels that read a known number of bytes no cache can hold:
  fetch_scale = known bytes / (FETCH_SIZE * 1024)
from k_calib_gather64w (64-byte rows, the 64 lanes of a wave in one table
window: the fixed-base gather pattern) for the table-gather kernels, and from
k_calib_stream (16 B per lane, coalesced) for the others.  WRITE_SIZE is used
as measured.

    python tools/pmc_r02.py <fetch_dir> <write_dir> <calib_dir> <calib.json> <bench.json> <R> <out.json> [valu_dir]

With valu_dir (the SQ_* pass), each entry also carries the per-launch VALU
instruction counts (INT32 / INT64 split, SQ_INSTS_VALU_MFMA_MOPS_F16 = 0: no
MFMA) and the derived VALUBusy (% of the launch's GPU time with VALU
instructions issuing, per CU) and SIMD_UTILIZATION.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GATHER = {"k_rp_fixed_exact", "k_rp_fixed_all", "k_rp_terms_fixed", "k_pv_fbsum", "k_sig_fixed", "k_token_open"}


def kernel_key(name):
    """'void fts::k_rp_fixed_exact<22>(...)' -> 'k_rp_fixed_exact' (the library's timing name)"""
    k = name.split("(")[0].replace("fts::", "")
    if k.startswith("void "):
        k = k[5:]
    return k.split("<")[0].strip()


def per_kernel(d, counter):
    acc = defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"])):
                if r["Counter_Name"] == counter:
                    acc[kernel_key(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def main():
    fdir, wdir, cdir, cjson, bjson, R, dst = sys.argv[1:8]
    R = int(R)
    known = json.load(open(cjson))
    cal = per_kernel(cdir, "FETCH_SIZE")
    scale = {}
    calib = {}
    for k, b in known.items():
        if k.startswith("k_calib_store"):  # WRITE_SIZE calibration (pmc_calib_write pass)
            continue
        v = cal.get(k)
        if v:
            fs = sum(v) / len(v) * 1024
            scale[k] = b / fs
            calib[k] = {"known_bytes": b, "fetch_size_bytes": round(fs), "scale": round(b / fs, 4)}
    bench = json.load(open(bjson))
    proofs = bench["isolated_pass"]["proofs"]
    batch = bench["config"]["batch_per_gpu"]
    # kernels that only the lone batch runs (passes <= FTS_COM_FIXED_MAX take the
    # latency path): their last dispatches are the isolated single batch
    LATENCY_ONLY = {"k_rp_fixed_all", "k_rp_xd", "k_rp_com_tree"}
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    vdir = sys.argv[8] if len(sys.argv) > 8 else None
    # raw SQ counts and the derived VALU-busy / SIMD-utilisation metrics of the pass
    SQ = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
          "SQ_INSTS_VALU_MFMA_MOPS_F16", "VALUBusy", "SIMD_UTILIZATION")
    valu = {c: per_kernel(vdir, c) for c in SQ} if vdir else {}
    out = {"_calibration": calib, "_source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs) of bench.py, "
                                             "last %d dispatches per kernel = the isolated pass of %d proofs"
                                             % (R, proofs)}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, [])[-R:], write.get(k, [])[-R:]
        e = {"dispatches": len(f)}
        if f:
            e["fetch_bytes"] = round(sum(f) / len(f) * 1024)
            e["fetch_scale"] = round(scale.get("k_calib_gather64w" if k in GATHER else "k_calib_stream", 1.0), 4)
        if w:
            e["write_bytes"] = round(sum(w) / len(w) * 1024)
        for c, per in valu.items():
            v = per.get(k, [])[-R:]
            if v:
                e[c] = round(sum(v) / len(v), 4) if c in ("VALUBusy", "SIMD_UTILIZATION") else round(sum(v) / len(v))
        out["%s@pass%d" % (k, batch if k in LATENCY_ONLY and proofs > batch else proofs)] = e
    print(json.dumps(calib))
    # the batch check's MSM sort (digits / two-level counting sort): bytes written per pass
    SORT = ("k_msm_digits", "k_msm_split", "k_rs_hist", "k_rs_pscan", "k_rs_pbase", "k_rs_scatter", "k_rs_part",
            "k_msm_scatter", "k_msm_local_sort")
    sw = sum(out[k].get("write_bytes", 0) for k in out if k.split("@")[0] in SORT and k.endswith("@pass%d" % proofs))
    out["_msm_sort_write_bytes@pass%d" % proofs] = sw
    print("msm sort kernels write %.3f GB per pass" % (sw / 1e9))
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k in ("k_rp_fixed_exact", "k_rp_fixed_all", "k_msm_chunks"):
        key = "%s@pass%d" % (k, proofs)
        if key in out:
            print(key, out[key])


if __name__ == "__main__":
    main()
