"""Per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch (bytes) from two
separate rocprofv3 --pmc passes of one command (tools/gpu_session.sh
identity_pmc).  FETCH_SIZE and WRITE_SIZE are reported in KiB by rocprofv3 on
gfx950; fetch bytes are given raw and x2 (the guide's factor for 16-B
coalesced streams, which the identity kernels' [word][lane] scratch and stack
accesses are; tools/fetch_calib measures both patterns).
    python tools/pmc_kernels.py <fetch_dir> <write_dir> <out.json> [kernel-substring ...]"""
import json
import sys

from pmc_traffic import per_kernel


def main():
    fdir, wdir, dst = sys.argv[1:4]
    keep = sys.argv[4:]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    out = {"_source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs), average per dispatch"}
    for k in sorted(set(fetch) | set(write)):
        if keep and not any(s in k for s in keep):
            continue
        f, w = fetch.get(k, []), write.get(k, [])
        e = {"dispatches": max(len(f), len(w))}
        if f:
            e["fetch_bytes_raw"] = round(sum(f) / len(f) * 1024)
            e["fetch_bytes_x2"] = 2 * e["fetch_bytes_raw"]
        if w:
            e["write_bytes"] = round(sum(w) / len(w) * 1024)
        out[k] = e
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, e in out.items():
        if not k.startswith("_"):
            print(k, e)


if __name__ == "__main__":
    main()
