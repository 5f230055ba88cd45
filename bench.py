"""Benchmark: range-proof verifies/sec (BN254, 64-bit) on MI355X.

Workload (BASELINE.json configs[1]): batches of 4,096
standalone 64-bit Bulletproof range proofs (synthetic, seeded 0xF7A50002 +
rank, produced by the library's host prover).  One step = one pass of the
hot path over one batch: fts_rp_batch_verify on a batch already resident in
HBM, verdicts delivered to the host; for N > 1 the per-GPU verdict bitmaps
are all-gathered over RCCL (the only exchange step).  Weak
scaling: every rank verifies its own 4,096-proof batch.

Other BASELINE.json configs as extra workloads (not the default line):
  --workload msm       configs[2] / C3: one BN254 G1 MSM over 2^--msm-log points
                       (fts_msm_run on staged inputs), terms/s
  --workload transfer  configs[3] / C4 per GPU: --transfers 2-in/2-out 64-bit
                       transfers (TypeAndSum + 2 rp64 each) per step through
                       fts_transfer_verify_batch, transfers/s
  --workload mixed     configs[4] / C5 per GPU: issues with 16 outputs and
                       2-in/2-out transfers (1 : 4) at 32-bit range, 1 % tampered,
                       one fts_actions_verify_batch per step, actions/s

Prints one JSON line (rank 0).  Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--bits 64]
  python bench.py --workload msm --msm-log 20
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import os

# Hardware queues per process: every lane uses two streams, and streams that
# share a HIP hardware queue serialise (the box's default is 4).  Read once at
# HIP runtime load, so raised here before anything loads HIP (DESIGN.md §5,
# lane sweep: 8 lanes run 2.4x faster with 16 queues than with 4).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))

# INT32 VALU peak of one MI355X for v_mad_u64_u32 (quarter rate):
# 256 CU x 4 SIMD x 32 lanes / 4 x 2.4 GHz (MI355X_MICROARCH.md chip table);
# tools' int_peak microbenchmark measures >= 88 % of it with the Fp product.
PEAK_TMAD = 256 * 4 * 32 / 4 * 2.4e9 / 1e12
R_ORDER = 21888242871839275222246405745257275088548364400416034343698204186575808495617
MAD_PER_MUL = 136          # 8x32-bit no-carry CIOS / FIPS Montgomery product
SURVEY_MAD_PER_RP64 = 8.13e6   # SURVEY §8(d) fixed cost model per rp64 verify


def _cpu_env():
    """host CPU model, logical CPUs and the cgroup CPU quota (the cores a baseline may use)"""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "cgroup_cpu_quota": quota}


def _lib_record():
    """which libfts_gpu.so this run loaded: its sha256, mtime and the record
    __graft_entry__.build() left (compiled by that call, or found up to date)"""
    import hashlib
    so = os.path.join(ROOT, "fabric-token-sdk_amd", "lib", "libfts_gpu.so")
    rec = {}
    try:
        with open(os.path.join(ROOT, "fabric-token-sdk_amd", "lib", "build_info.json")) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        rec = {"build_info": "absent (library not built by __graft_entry__.build())"}
    try:
        with open(so, "rb") as f:
            dg = hashlib.sha256(f.read()).hexdigest()
        rec["loaded_so_sha256"] = dg[:16]
        rec["matches_build_record"] = dg == rec.get("so_sha256")
        rec["so_mtime"] = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(os.path.getmtime(so)))
    except OSError:
        pass
    rec.pop("so_sha256", None)
    return rec


# the reference-order C restatement beside the reference's own Go verifier
PORT_NOTE = ("portable 4x64-bit Montgomery C (no GLV, no assembly, affine G1.Mul as bulletproof.go/ipa.go call "
             "them); the reference's gnark-crypto uses assembly Montgomery products and GLV, so a Go run of the "
             "reference would likely be 2-4x faster per core than this column (unmeasured: no Go toolchain here)")


def _timed_sample(fn, total, chunk, seconds):
    """run fn(lo, hi) over chunks of [0, total) until `seconds` of wall time; -> (items, s)"""
    done, cs = 0, 0.0
    while cs < seconds and done < total:
        c = min(chunk, total - done)
        t0 = time.perf_counter()
        fn(done, done + c)
        cs += time.perf_counter() - t0
        done += c
    return done, cs


def _cpu_batch_baseline(opp, coms, proofs, want, thr, args):
    """SURVEY 8(d)'s "optimized CPU batch" column: the device's batch algorithm
    (fixed-base tables, GLV com chain, one RLC + Pippenger MSM per batch;
    oracle/c/cpu_batch.c) on host threads, over the same proofs.  Tables are built
    before the clock.  -> dict for cpu_baseline["optimized_batch"]"""
    from oracle import cref
    W = 13
    t = time.perf_counter()
    cb = cref.CpuBatch(opp, W, thr)
    setup = time.perf_counter() - t
    nfb = [0]

    def run(lo, hi, t):
        got, f = cb.verify(coms[lo:hi], proofs[lo:hi], threads=t)
        nfb[0] += f
        assert got == [int(w) for w in want[lo:hi]], "optimized CPU batch verdicts differ"
    B = len(proofs)
    d1, s1 = _timed_sample(lambda lo, hi: run(lo, hi, 1), B, 256, args.cpu_seconds / 4)
    dn, sn = _timed_sample(lambda lo, hi: run(lo, hi, thr), B, B, args.cpu_seconds)
    cb.close()
    return {"value": round(dn / sn, 1), "value_1core": round(d1 / s1, 1), "cores": thr, "kind": "port",
            "sample": "%d proofs in batches of %d (%d threads) and %d in batches of 256 (1 thread), the same proofs; "
                      "oracle/c/cpu_batch.c: %d-bit signed-window fixed-base tables (built in %.1f s, untimed), "
                      "GLV/Straus com chain, one RLC + GLV Pippenger MSM per batch, bisection on failure; "
                      "4x64-bit Montgomery C (no assembly); %.1f + %.1f s wall, %d proofs took the per-proof fallback"
                      % (dn, min(B, dn), thr, d1, W, setup, sn, s1, nfb[0])}


def _action_cpu_baseline(pp_raw, bits, actions, want, args, unit, what):
    """reference-order C restatement of transfer / issue Verify (oracle/c/ref_verify.c
    oracle_action_verify_many) on a bounded sample of the same actions: 1 core, then
    --cpu-threads cores; verdicts checked against `want` [(status, fail index)]"""
    from oracle import cref, pp as oppm
    opp = oppm.load_pp(pp_raw).with_bit_length(bits)
    thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))

    def run(lo, hi, t):
        got = cref.action_verify_many(opp, actions[lo:hi], threads=t)
        assert got == want[lo:hi], "CPU oracle verdicts differ"
    d1, s1 = _timed_sample(lambda lo, hi: run(lo, hi, 1), len(actions), 2, args.cpu_seconds / 3)
    dn, sn = _timed_sample(lambda lo, hi: run(lo, hi, thr), len(actions), 4 * thr, args.cpu_seconds)
    cpu = {"value": round(dn / sn, 3), "unit": unit, "cores": thr, "kind": "port", "value_1core": round(d1 / s1, 3),
           "sample": "%d (%d threads) and %d (1 thread) of the same %s, reference-order C restatement of "
                     "transfer/issue Verify (oracle/c/ref_verify.c oracle_action_verify_many: TypeAndSum / "
                     "SameType + RangeCorrectness, affine G1.Mul per operation), %.1f + %.1f s wall"
                     % (dn, thr, d1, what, sn, s1)}
    cpu.update(_cpu_env())
    return cpu


def _cg_throttle():
    """(nr_throttled, throttled_usec) of this process's cgroup (v2), if readable"""
    try:
        d = dict(l.split() for l in open("/sys/fs/cgroup/cpu.stat"))
        return int(d["nr_throttled"]), int(d["throttled_usec"])
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=64)
    ap.add_argument("--inflight", type=int, default=64,
                    help="batches in flight: host threads, each submitting its own staged batch")
    ap.add_argument("--lanes", type=int, default=int(os.environ.get("FTS_LANES", "4")),
                    help="device lanes (stream pairs) of the library (FTS_LANES); batches submitted while "
                         "all lanes are busy are coalesced into one device pass (FTS_COALESCE_MAX proofs)")
    ap.add_argument("--distinct", type=int, default=64,
                    help="batches with distinct proofs (default: every in-flight batch, so every pass -- and the "
                         "isolated roofline pass -- holds distinct proofs); the other in-flight batches re-stage them")
    ap.add_argument("--pass-batches", type=int, default=0,
                    help="batches in the isolated roofline pass (0: FTS_COALESCE_MAX / batch, the pass size the "
                         "library runs under load; the PMC traffic file is keyed by this pass size)")
    ap.add_argument("--roofline-steps", type=int, default=6,
                    help="isolated steps (one batch alone on the GPU) for the per-kernel roofline")
    ap.add_argument("--tamper-every", type=int, default=1,
                    help="with --tamper: tamper only every M-th staged batch (e.g. --tamper 1e-9 --tamper-every 20: "
                         "one bad proof per 81,920-proof pass)")
    ap.add_argument("--tamper", type=float, default=0.0,
                    help="rp workload: fraction of tampered proofs per batch (SURVEY 8d: the C2 variant with 1 %% "
                         "tampered proofs exercises the group-test fallback); verdicts are checked every step")
    ap.add_argument("--cpu-sample", type=int, default=256, help="CPU baseline chunk size (0: skip the CPU baseline)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--host-steps", type=int, default=64,
                    help="rp workload: calls of fts_rp_verify_batch from host DER bytes after the timed region "
                         "(the PCIe-inclusive rate, reported apart; 0: skip)")
    ap.add_argument("--host-inflight", type=int, default=16,
                    help="rp workload: host threads calling fts_rp_verify_batch concurrently for host_inclusive")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="wall-time bound of the CPU baseline sample")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic per launch (tools/pmc_traffic.py); default: the newest profiles/traffic_rNN.json")
    ap.add_argument("--workload", choices=["rp", "msm", "transfer", "mixed", "request", "audit", "prove", "ecdsa",
                                           "idemix", "identity"],
                    default="rp")
    ap.add_argument("--sigs", type=int, default=65536, help="ecdsa workload: owner signatures per GPU per step")
    ap.add_argument("--msg-len", type=int, default=1024, help="ecdsa / idemix workloads: signed message bytes")
    ap.add_argument("--idemix-curve", choices=["bn254", "fp256bn"], default="bn254",
                    help="idemix workload: issuer key curve (bn254: the key of zkatdlog_pp.json; "
                         "fp256bn: the validator tests' key)")
    ap.add_argument("--tokens", type=int, default=65536, help="audit workload: token openings per GPU per step")
    ap.add_argument("--prove-kind", choices=["rp", "transfer"], default="rp",
                    help="prove workload: standalone range proofs, or whole 2-in/2-out transfers")
    ap.add_argument("--msm-log", type=int, default=20, help="msm workload: log2 of the point count")
    ap.add_argument("--msm-tiled", action="store_true",
                    help="msm workload: 2^16 distinct points tiled (rounds 2-3) instead of 2^msm-log distinct ones")
    ap.add_argument("--transfers", type=int, default=8192, help="transfer/mixed workloads: transfers per GPU per step")
    ap.add_argument("--action-inflight", type=int, default=None,
                    help="concurrent verify calls (host threads) of the non-C2 workloads; default 8 for the "
                         "action workloads (transfer / mixed / request: the library coalesces concurrent calls "
                         "into shared passes, as a validator's goroutines would submit them), 3 otherwise")
    args = ap.parse_args()
    if args.action_inflight is None:
        args.action_inflight = (8 if args.workload in ("transfer", "mixed", "request")
                                else 8 if args.workload == "identity" else 3)
    if args.workload == "msm":
        return bench_msm(args)
    if args.workload == "transfer":
        return bench_transfer(args)
    if args.workload == "mixed":
        return bench_mixed(args)
    if args.workload == "ecdsa":
        return bench_ecdsa(args)
    if args.workload == "idemix":
        return bench_idemix(args)
    if args.workload == "identity":
        return bench_identity(args)
    if args.workload == "audit":
        return bench_audit(args)
    if args.workload == "prove":
        return bench_prove(args)
    if args.workload == "request":
        return bench_transfer(args, raw_requests=True)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FTS_DIST_BACKEND=gloo + FTS_DEVICE=0 rehearse the N > 1 path with every
    # rank on one GPU (the exchange then runs over CPU tensors)
    backend = os.environ.get("FTS_DIST_BACKEND", "nccl")
    local = int(os.environ.get("FTS_DEVICE", str(local)))
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    os.environ["FTS_LANES"] = str(max(1, args.lanes))
    import random
    import numpy as np
    import fts_gpu
    from fts_gpu import dist as fdist

    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=args.bits, device=local)
    pp.reserve()  # every lane's workspace sized for the largest coalesced pass, before the clock
    n, k, B = pp.bit_length, pp.rounds, args.batch
    # one staged batch per in-flight slot; the first `distinct` hold distinct
    # proofs, the rest re-stage them (verification work does not depend on it)
    inflight = max(1, args.inflight)
    t0 = time.time()
    batches, sets, wants, staged = [], [], [], []
    for ln in range(inflight):
        if ln >= max(1, args.distinct):
            proofs, coms = sets[ln % len(sets)]
        else:
            rng = random.Random(fdist.shard_seed(0xF7A50002, rank, ln))
            vals = [rng.getrandbits(n) for _ in range(B)]
            bfs = [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(B)]
            # device prover: byte-identical to the host prover (tests/test_gpu_prove.py), seconds faster
            proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=0xF7A50002 + 1000003 * rank + 7777 * ln)
            sets.append((proofs, coms))
        want = np.zeros(B, dtype=np.int32)
        if args.tamper > 0 and ln % max(1, args.tamper_every) == 0:
            # T1 (-> invalid range proof) or one L_j (-> invalid IPA), before the clock
            from oracle import bn254 as obn, zkat
            proofs = list(proofs)
            trng = random.Random(0x7A3 + 31 * ln + 7919 * rank)
            for i in trng.sample(range(B), max(1, round(args.tamper * B))):
                r = zkat.RangeProof.deserialize(proofs[i])
                if trng.random() < 0.5:
                    r.data.T1 = obn.g1_add(r.data.T1, obn.GEN)
                    want[i] = fts_gpu.FTS_E_RP_INVALID
                else:
                    j = trng.randrange(k)
                    r.ipa.L[j] = obn.g1_add(r.ipa.L[j], obn.GEN)
                    want[i] = fts_gpu.FTS_E_IPA_INVALID
                proofs[i] = r.serialize()
        wants.append(want)
        staged.append((proofs, coms))
        batches.append(pp.stage_range_proofs(proofs, coms))
    proofs0, coms0 = staged[0]  # batch 0 (tampered when --tamper is given; its verdicts are wants[0])
    prove_s = time.time() - t0

    def run(ln, nsteps, sink):
        for _ in range(nsteps):
            st = batches[ln].verify(want_status=True)
            sink.append((st, batches[ln].merged()))
            if args.tamper > 0:
                assert (st == wants[ln]).all(), "verdicts differ from the tampered positions"

    def pipelined(nsteps, on_ready=None):
        """nsteps batch verifications spread over the in-flight slots (one host
        thread each); for N > 1 every step's verdict bitmap is all-gathered.
        The submitter threads are created first and released together through
        a barrier, so the timed region starts when the K steps are submitted
        (not while Python spawns threads one by one).  on_ready runs once every
        submitter waits at the gate, before the clock starts.  -> (res, t0)"""
        per = [nsteps // inflight + (1 if i < nsteps % inflight else 0) for i in range(inflight)]
        active = [i for i in range(inflight) if per[i] > 0]
        sinks = [[] for _ in range(inflight)]
        gate = threading.Barrier(len(active) + 1)

        def body(i):
            gate.wait()
            run(i, per[i], sinks[i])
        th = [threading.Thread(target=body, args=(i,)) for i in active]
        for t in th:
            t.start()
        if on_ready is not None:
            on_ready()
        t0 = time.perf_counter()
        gate.wait()
        for t in th:
            t.join()
        res = [x for s in sinks for x in s]
        if dist is not None:
            for st, _ in res:
                fdist.allgather_verdicts(dist, st)
        return res, t0

    # warmup in the timed region's shape: bursts of `steps` submissions while that is
    # fewer than the in-flight slots (the driver's 20-step line), else one stream
    warm = max(args.warmup, inflight)
    if args.steps < inflight:
        for _ in range(-(-warm // args.steps)):
            pipelined(args.steps)
    else:
        pipelined(warm)

    def before_timed():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()
    cg0, cpu0 = _cg_throttle(), time.process_time()
    res, t0 = pipelined(args.steps, on_ready=before_timed)
    if dist is not None:
        import torch
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host = {"cpu_s": round(time.process_time() - cpu0, 3), "wall_s": round(elapsed, 3)}
    cg1 = _cg_throttle()
    if cg0 and cg1:
        host["cgroup_throttled_periods"] = cg1[0] - cg0[0]
        host["cgroup_throttled_ms"] = round((cg1[1] - cg0[1]) / 1e3, 1)
    ok = int(sum(int((st == 0).sum()) for st, _ in res))  # verdicts of the timed steps
    merged_avg = sum(m for _, m in res) / max(1, len(res))
    if dist is not None:
        elapsed = fdist.reduce_scalar(dist, elapsed, "max")
        ok = int(fdist.reduce_scalar(dist, ok, "sum"))

    total = world * B * args.steps
    value = total / elapsed

    # Isolated passes (after the timed region), so each kernel's HIP-event
    # time is its own (in the pipelined region kernels of several passes share
    # the CUs and their event spans overlap):
    #  1. one 4,096-proof batch alone: the single-batch latency view;
    #  2. one pass of the size the timed region ran (merged_batches_avg
    #     batches, coalesced), alone: the ROOFLINE launch -- run last, so the
    #     last R dispatches of a rocprofv3 trace / PMC pass are exactly these.
    R = max(1, args.roofline_steps)

    def isolated(batch, reps, want):
        acc = {}
        t = time.perf_counter()
        for _ in range(reps):
            st = batch.verify(want_status=True)
            assert (st == want).all()
            for name, (ms, mads) in batch.timings().items():
                o = acc.get(name, (0.0, 0.0))
                acc[name] = (o[0] + ms, mads)
        return acc, (time.perf_counter() - t) * 1e3 / reps

    kt1, iso_ms = isolated(batches[0], R, wants[0])
    m = args.pass_batches or max(1, int(os.environ.get("FTS_COALESCE_MAX", "81920")) // B)
    pass_proofs = [staged[i % len(staged)] for i in range(m)]
    big = pp.stage_range_proofs([p for ps, _ in pass_proofs for p in ps], [c for _, cs in pass_proofs for c in cs])
    kt, pass_ms = isolated(big, R, np.concatenate([wants[i % len(wants)] for i in range(m)]))
    big.close()
    avg = {kname: v[0] / R for kname, v in kt.items()}
    avg1 = {kname: v[0] / R for kname, v in kt1.items()}
    # roofline kernel: the largest share of the algorithmic work (MADs/launch);
    # the longest (latency-bound) kernel is reported beside it
    dom = max(kt, key=lambda kname: kt[kname][1])
    dom1 = max(kt1, key=lambda kname: kt1[kname][1])  # a lone batch may take the latency path's kernels
    longest = max((kn for kn in avg if not kn.startswith("host_")), key=avg.get)

    def kernel_roof(kname):
        ms, mads = avg[kname], kt[kname][1]
        ach = mads / (ms * 1e-3) / 1e12 if mads and ms > 0 else None
        return {"kernel": kname, "kernel_ms": round(ms, 4), "mads_per_launch": mads,
                "achieved": round(ach, 3) if ach else None, "frac": round(ach / PEAK_TMAD, 4) if ach else None}

    # this pipeline's own cost model: algorithmic MADs of every kernel of one pass / proofs
    own_mads = sum(v[1] for v in kt.values()) / (m * B)
    traffic = None
    tj_path = args.traffic_json
    if tj_path is None:
        import glob
        cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_r[0-9][0-9].json")))
        tj_path = cands[-1] if cands else ""
    try:
        with open(tj_path) as f:
            tj = json.load(f)
            # HBM bytes per launch of THIS pass size: FETCH_SIZE (scaled by the factor calibrated for the
            # kernel's access pattern, tools/fetch_calib) + WRITE_SIZE, from separate PMC runs of the same command
            e = tj.get("%s@pass%d" % (dom, m * B), {})
            if e.get("fetch_bytes") is not None:
                traffic = int(e["fetch_bytes"] * e.get("fetch_scale", 1.0) + e.get("write_bytes", 0))
    except (OSError, ValueError, AttributeError):
        pass
    rd = kernel_roof(dom)
    roofline = {"bound": "int32_valu (v_mad_u64_u32)", "kernel": dom, "achieved": rd["achieved"],
                "peak": round(PEAK_TMAD, 3), "unit": "TMAD/s", "frac": rd["frac"], "traffic": traffic,
                "traffic_source": os.path.basename(tj_path) if traffic is not None else None,
                "kernel_ms": rd["kernel_ms"], "mads_per_launch": rd["mads_per_launch"],
                "measured": "HIP events, %d isolated passes of %d proofs (%d coalesced batches, the timed region's "
                            "pass size) alone on the GPU after the timed region" % (R, m * B, m),
                "pipeline_frac_survey_model": round(value / world * SURVEY_MAD_PER_RP64 / (PEAK_TMAD * 1e12), 4),
                "pipeline_mads_per_rp64": round(own_mads),
                "pipeline_frac_own_model": round(value / world * own_mads / (PEAK_TMAD * 1e12), 4)}
    longest_kernel = kernel_roof(longest)

    # the drop-in boundary from host buffers, after the timed region: DER bytes in
    # (fts_rp_verify_batch: host parse + upload + verify + verdicts back), the
    # PCIe-inclusive rate a Go caller without staged batches sees; not `value`
    host_inclusive = None
    if rank == 0 and args.host_steps > 0:
        from fts_gpu import _lib as FL, _ptr_array
        _bufs, ptrs, lens = _ptr_array(proofs0)
        comsb = b"".join(coms0)

        class HostStep:
            @staticmethod
            def verify():
                st = np.zeros(B, dtype=np.int32)
                FL.check("fts_rp_verify_batch", FL.lib.fts_rp_verify_batch(
                    pp._ctx, B, ptrs, lens, comsb, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
                assert (st == wants[0]).all()
                return st
        hs = [HostStep() for _ in range(max(1, min(args.host_inflight, args.host_steps)))]
        _run_action_steps(hs, len(hs), None, None)  # warm the host pool
        h_el, _ = _run_action_steps(hs, args.host_steps, None, None)
        host_inclusive = {"value": round(B * args.host_steps / h_el, 1), "unit": "verifies/s",
                          "ms_per_step": round(h_el / args.host_steps * 1e3, 4), "steps": args.host_steps,
                          "inflight": len(hs),
                          "note": "fts_rp_verify_batch from host DER bytes (parse + H2D + verify + D2H), %d calls "
                                  "from %d host threads, after the timed region" % (args.host_steps, len(hs))}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        # bounded samples of the same proofs: one core, then --cpu-threads cores
        from oracle import cref, pp as oppm
        opp = oppm.load_pp(pp_raw).with_bit_length(n)
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))

        def chk(lo, hi, t):
            res = cref.rp_verify_many(opp, coms0[lo:hi], proofs0[lo:hi], threads=t)
            assert res == [int(w) for w in wants[0][lo:hi]], res
        d1, s1 = _timed_sample(lambda lo, hi: chk(lo, hi, 1), B, 8, args.cpu_seconds / 3)
        dn, sn = _timed_sample(lambda lo, hi: chk(lo, hi, thr), B, max(thr, args.cpu_sample), args.cpu_seconds)
        cpu = {"value": round(dn / sn, 3), "unit": "rp%d verifies/s" % n, "cores": thr, "kind": "port",
               "value_1core": round(d1 / s1, 3),
               "sample": "%d (%d threads) and %d (1 thread) of the same rp%d proofs, reference-order C restatement "
                         "(oracle/c/ref_verify.c, %d affine G1.Mul per proof, no GLV / assembly), %.1f + %.1f s wall"
                         % (dn, thr, d1, n, 7 * n + 2 * k + 9, sn, s1),
               "vs_reference_go": PORT_NOTE}
        cpu["optimized_batch"] = _cpu_batch_baseline(opp, coms0, proofs0, wants[0], thr, args)
        cpu.update(_cpu_env())

    if rank == 0:
        out = {
            "metric": "range-proof verifies/sec (BN254, %d-bit)" % n,
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: %d seeded %d-bit range proofs per batch from the library's device prover "
                    "(byte-identical to its host prover), %d distinct batches (%d distinct proofs)"
                    % (B, n, min(inflight, max(1, args.distinct)), B * min(inflight, max(1, args.distinct))),
            "config": {"workload": "C2: batch of %d standalone %d-bit Bulletproof range proofs per GPU "
                                   "(exact transcripts per proof + RLC batch check via one Pippenger MSM)%s"
                                   % (B, n, _tamper_note(args, B)),
                       "batch_per_gpu": B, "bit_length": n, "rounds": k, "parallelism": "shard%d" % world},
            "accepted": ok,
            "verified": world * B * args.steps,
            "inflight": inflight,
            "device_lanes": args.lanes,
            "merged_batches_avg": round(merged_avg, 2),
            "host": host,
            "isolated_batch": {"ms": round(iso_ms, 3), "verifies_per_s": round(B / iso_ms * 1e3, 1),
                               "note": "one %d-proof batch alone on the GPU (latency; no coalescing)" % B,
                               "roofline_kernel": dom1,
                               "roofline_kernel_ms": round(avg1.get(dom1, 0.0), 4),
                               "roofline_frac": round(kt1[dom1][1] / (avg1[dom1] * 1e-3) / 1e12 / PEAK_TMAD, 4)
                               if avg1.get(dom1) else None},
            "isolated_pass": {"proofs": m * B, "ms": round(pass_ms, 3), "verifies_per_s": round(m * B / pass_ms * 1e3, 1)},
            "host_inclusive": host_inclusive,
            "roofline": roofline,
            "longest_kernel": longest_kernel,
            "cpu_baseline": cpu,
            "kernel_ms_isolated": {kname: round(v, 4) for kname, v in avg.items()},
            "tampered": args.tamper,
            "tamper_every": args.tamper_every,
            "fallback": _fallback_share(kt, R, pass_ms),
            "prove_s": round(prove_s, 2),
            "library": _lib_record(),
            # fixed-base tables resident in HBM: 16-bit windows for the 2n + 6 public
            # generators, 20- or 22-bit (the default where the memory allows) for H_i, K, P
            "table_bytes": pp.table_bytes,
            "wide_table_bits": pp.wide_bits,
            "distinct_batches": min(inflight, max(1, args.distinct)),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# ------------------------------------------------------------- extra workloads
def _dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FTS_DIST_BACKEND=gloo + FTS_DEVICE=0 rehearse the N > 1 path with every
    # rank on one GPU (the exchange then runs over CPU tensors)
    backend = os.environ.get("FTS_DIST_BACKEND", "nccl")
    local = int(os.environ.get("FTS_DEVICE", str(local)))
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local, dist


def _max_over_ranks(dist, x):
    if dist is None:
        return x
    from fts_gpu import dist as fdist
    return fdist.reduce_scalar(dist, x, "max")


def _seq_points(m):
    """P_i = (i+1) G for i < m (affine, successive additions; synthetic input)"""
    p, G = 21888242871839275222246405745257275088696311157297823662689037894645226208583, (1, 2)
    out, (x, y) = [], G
    out.append((x, y))
    for _ in range(m - 1):
        if x == G[0]:
            lam = 3 * x * x * pow(2 * y, -1, p) % p
        else:
            lam = (y - G[1]) * pow(x - G[0], -1, p) % p
        x3 = (lam * lam - x - G[0]) % p
        y = (lam * (x - x3) - y) % p
        x = x3
        out.append((x, y))
    return out


def _mul_g(k, base=(1, 2)):
    """k P (double-and-add, affine; P = G by default; used once to check the MSM result)"""
    p = 21888242871839275222246405745257275088696311157297823662689037894645226208583
    acc = None
    while k:
        if k & 1:
            acc = base if acc is None else _add(acc, base, p)
        base = _add(base, base, p)
        k >>= 1
    return acc


def _add(a, b, p):
    if a[0] == b[0]:
        if (a[1] + b[1]) % p == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, p) % p
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, p) % p
    x3 = (lam * lam - a[0] - b[0]) % p
    return (x3, (lam * (a[0] - x3) - a[1]) % p)


def _roofline_from(timings, steps):
    """dominant kernel (largest algorithmic MAD count) of the per-kernel timings
    (the batch check's fallback kernels, "fb:" names, are reported apart)"""
    dom = max((k for k in timings if not k.startswith("fb:")), key=lambda k: timings[k][1])
    ms, mads = timings[dom][0] / steps, timings[dom][1]
    ach = mads / (ms * 1e-3) / 1e12 if mads and ms > 0 else None
    return {"bound": "int32_valu (v_mad_u64_u32)", "kernel": dom, "achieved": round(ach, 3) if ach else None,
            "peak": round(PEAK_TMAD, 3), "unit": "TMAD/s", "frac": round(ach / PEAK_TMAD, 4) if ach else None,
            "traffic": None, "kernel_ms": round(ms, 4), "mads_per_launch": mads}


def _msm_roofline(kt, args):
    """C3 roofline, with PMC HBM bytes per launch of the dominant kernel and of the
    sort kernels from the newest profiles/msm22_traffic_rNN.json (tools/gpu_session.sh
    msm_pmc: FETCH_SIZE + WRITE_SIZE, separate runs of this workload at 2^22 points)"""
    roof = _roofline_from(kt, args.steps)
    if args.msm_log != 22 or args.msm_tiled:
        return roof
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "msm22_traffic_r[0-9][0-9].json")))
    if not cands:
        return roof
    try:
        with open(cands[-1]) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return roof

    def tb(k):
        e = tj.get(k) or {}
        return None if e.get("fetch_bytes_raw") is None else e["fetch_bytes_raw"] + e.get("write_bytes", 0)
    roof["traffic"] = tb(roof["kernel"])
    roof["traffic_source"] = os.path.basename(cands[-1])
    roof["traffic_per_kernel"] = {k: tb(k) for k in tj if not k.startswith("_") and tb(k) is not None}
    return roof


def _run_action_steps(batches, steps, dist, gather):
    """`steps` verify() calls spread over one host thread per prepared batch
    (concurrent calls run on different device lanes, so one call's host DER
    parsing overlaps another's kernels); returns (elapsed, per-kernel timings)"""
    per = [steps // len(batches) + (1 if i < steps % len(batches) else 0) for i in range(len(batches))]
    outs = [[] for _ in batches]

    def run(i):
        for _ in range(per[i]):
            outs[i].append(batches[i].verify())

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(batches))]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        for o in outs:
            for r in o:
                gather(r)
    return elapsed, outs


def bench_msm(args):
    world, rank, local, dist = _dist_setup()
    import random
    import fts_gpu
    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=args.bits, device=local)
    n = 1 << args.msm_log
    t0 = time.time()
    rng = random.Random(0xF7A50003 + rank)
    ks = [rng.randrange(R_ORDER) for _ in range(n)]
    scs = b"".join(k.to_bytes(32, "big") for k in ks)
    if args.msm_tiled:
        # round-2/3 input: 2^16 distinct points (i + 1) G tiled n / 2^16 times (L2-resident)
        m = min(n, 1 << 16)
        base = b"".join(x.to_bytes(32, "big") + y.to_bytes(32, "big") for x, y in _seq_points(m))
        pts = base * (n // m)
        st = pp.stage_msm(pts, scs)
        data = "synthetic: P_i = (i mod 2^16 + 1) G (tiled), uniform scalars mod r (seed 0xF7A50003 + rank)"
        e = _mul_g(sum(k * (i % m + 1) for i, k in enumerate(ks)) % R_ORDER)
    else:
        # n DISTINCT points k'_i * ped1, uniform k'_i, generated on the device
        # (fts_msm_stage_multiples) from 32-byte BE k'_i; closed form (sum s_i k'_i) * ped1
        kp = [rng.randrange(R_ORDER) for _ in range(n)]
        st = pp.stage_msm_multiples(b"".join(k.to_bytes(32, "big") for k in kp), scs)
        c1 = pp.token_commit(b"C3", 1, bytes(32))
        c0 = pp.token_commit(b"C3", 0, bytes(32))
        P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
        a = (int.from_bytes(c1[:32], "big"), int.from_bytes(c1[32:], "big"))
        b_ = (int.from_bytes(c0[:32], "big"), (-int.from_bytes(c0[32:], "big")) % P)
        ped1 = _add(a, b_, P)
        pts = None
        data = "synthetic: 2^%d distinct points P_i = k'_i ped1 (uniform k'_i, made on the device), uniform " \
               "scalars mod r (seed 0xF7A50003 + rank)" % args.msm_log
        e = _mul_g(sum(k * q for k, q in zip(ks, kp)) % R_ORDER, ped1)
    setup_s = time.time() - t0
    for _ in range(max(1, args.warmup)):
        res = st.run()
    assert res == (bytes(64) if e is None else e[0].to_bytes(32, "big") + e[1].to_bytes(32, "big")), "MSM mismatch"
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    kt = {}
    for _ in range(args.steps):
        st.run()
        for name, (ms, mads) in st.timings().items():
            o = kt.get(name, (0.0, 0.0))
            kt[name] = (o[0] + ms, mads)
    elapsed = _max_over_ranks(dist, time.perf_counter() - t0)
    value = world * n * args.steps / elapsed
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from oracle import cref
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        # "the build's C++ Pippenger" -- oracle/c/cpu_batch.c's GLV
        # Pippenger (signed windows, threads over (window, part)) over the first
        # 2^min(L, 20) of the SAME points (downloaded from the device: fts_msm_points),
        # its result checked against the sample's closed form
        ns = min(n, 1 << 20)
        if pts is None:
            spts = st.points(0, ns)
            want_s = _mul_g(sum(k * q for k, q in zip(ks[:ns], kp[:ns])) % R_ORDER, ped1)
        else:
            spts = pts[:64 * ns]
            want_s = _mul_g(sum(k * (i % (1 << 16) + 1) for i, k in enumerate(ks[:ns])) % R_ORDER)
        want_b = bytes(64) if want_s is None else want_s[0].to_bytes(32, "big") + want_s[1].to_bytes(32, "big")
        reps, cs = 0, 0.0
        while reps == 0 or cs < args.cpu_seconds / 2:
            t1 = time.perf_counter()
            got = cref.msm_pippenger(spts, scs[:32 * ns], threads=thr)
            cs += time.perf_counter() - t1
            reps += 1
            assert got == want_b, "CPU Pippenger differs from the closed form"
        # the reference's own call pattern beside it: term-by-term G1.Mul + Add (ipa.go:254-259)
        done, ct = 0, 0.0
        while ct < args.cpu_seconds / 4 and done < ns:
            c = min(1024, ns - done)
            t1 = time.perf_counter()
            cref.msm(spts[64 * done:64 * (done + c)], scs[32 * done:32 * (done + c)], threads=thr)
            ct += time.perf_counter() - t1
            done += c
        cpu = {"value": round(reps * ns / cs, 1), "unit": "terms/s", "cores": thr, "kind": "port",
               "sample": "%d x the MSM over the first %d of the same points (GLV Pippenger, oracle/c/cpu_batch.c "
                         "cpu_msm_pippenger, portable 4x64 C), %d threads, %.1f s wall; result = the closed form"
                         % (reps, ns, thr, cs),
               "vs_reference_go": "gnark-crypto's MultiExp (assembly Montgomery, GLV, windowed Pippenger) would "
                                  "likely be 2-4x faster per core than this portable C (unmeasured: no Go here)",
               "term_by_term": {"value": round(done / ct, 1), "unit": "terms/s",
                                "sample": "%d terms, G1.Mul + Add per term (oracle/c/ref_verify.c oracle_msm, the "
                                          "reference's ipa.go:254-259 pattern), %d threads, %.1f s" % (done, thr, ct)}}
        cpu.update(_cpu_env())
    if rank == 0:
        print(json.dumps({
            "metric": "BN254 G1 MSM terms/sec (2^%d points)" % args.msm_log, "value": round(value, 1),
            "unit": "terms/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (BN254 Fp 8x32-bit Montgomery)",
            "data": data,
            "config": {"workload": "C3: standalone G1 MSM, 2^%d points per GPU (fts_msm_run, inputs resident in HBM)"
                                   % args.msm_log, "points": n, "parallelism": "shard%d" % world},
            "roofline": _msm_roofline(kt, args), "cpu_baseline": cpu,
            "kernel_ms": {k: round(v[0] / args.steps, 4) for k, v in kt.items()}, "setup_s": round(setup_s, 2)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_prove(args):
    """batched range-proof proving (rangeProver.Prove,
    bulletproof.go:209-249) on the device.  One step = one fts_rp_prove_batch_gpu
    over --batch proofs (host randomness draw + DER serialisation included)."""
    world, rank, local, dist = _dist_setup()
    import random
    import fts_gpu
    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=args.bits, device=local)
    if args.prove_kind == "transfer":
        return _bench_prove_transfers(args, pp, world, rank, dist)
    n = args.batch
    rng = random.Random(0xF7A500B0 + rank)
    vals = [rng.randrange(1 << args.bits) for _ in range(n)]
    bfs = [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(n)]
    proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=1)
    st = pp.verify_range_proofs(proofs, coms)
    assert int((st != 0).sum()) == 0, "device proofs rejected"
    for _ in range(max(0, args.warmup - 1)):
        pp.prove_range_batch_gpu(vals, bfs, seed=1)
    if dist is not None:
        dist.barrier()

    class Step:  # concurrent calls run on different device lanes: host work overlaps device work
        def __init__(self, i):
            self.i, self.s = i, 0

        def verify(self):
            self.s += 1
            return pp.prove_range_batch_gpu(vals, bfs, seed=1 + (self.i * 1000 + self.s) * n)

    elapsed, _ = _run_action_steps([Step(i) for i in range(max(1, args.action_inflight))], args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    kt = {}  # one call alone on the GPU (per-kernel view)
    reps = 2
    for s in range(reps):
        pp.prove_range_batch_gpu(vals, bfs, seed=1)
        for name, (ms, mads) in pp.last_timings_ex().items():
            o = kt.get(name, (0.0, 0.0))
            kt[name] = (o[0] + ms, mads)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        done, cs = 0, 0.0
        while cs < args.cpu_seconds and done < n:
            c = min(1024, n - done)
            t1 = time.perf_counter()
            h, _ = pp.prove_range_batch(vals[done:done + c], bfs[done:done + c], seed=1 + done, threads=thr)
            cs += time.perf_counter() - t1
            assert h[0] == proofs[done], "host and device proofs differ"
            done += c
        cpu = {"value": round(done / cs, 1), "unit": "rp64 proofs/s", "cores": thr, "kind": "port",
               "sample": "%d of the same proofs, the library's host prover (C++ restatement of rangeProver.Prove "
                         "with 16-bit fixed-base tables, byte-identical output), %d threads, %.1f s wall"
                         % (done, thr, cs)}
    if rank == 0:
        print(json.dumps({
            "metric": "range-proof proves/sec (BN254, %d-bit)" % args.bits, "value": round(value, 1),
            "unit": "proofs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: %d seeded values / blinding factors (seed 0xF7A500B0 + rank)" % n,
            "config": {"workload": "SURVEY 8f rank 2: %d range proofs per GPU per step via fts_rp_prove_batch_gpu, "
                                   "%d calls in flight" % (n, max(1, args.action_inflight)), "batch_per_gpu": n, "bit_length": args.bits,
                       "parallelism": "shard%d" % world},
            "roofline": _roofline_from(kt, reps), "cpu_baseline": cpu, "inflight": max(1, args.action_inflight),
            "kernel_ms": {k: round(v[0] / reps, 4) for k, v in kt.items()}}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _bench_prove_transfers(args, pp, world, rank, dist):
    """2-in/2-out transfers proven whole on the device (TypeAndSum + 2 range proofs each,
    fts_transfer_prove_batch_gpu), --transfers per step"""
    import random
    import fts_gpu
    rng = random.Random(0xF7A500B1 + rank)
    n = args.transfers
    trs = []
    for _ in range(n):
        a, b = rng.randrange(1 << 62), rng.randrange(1 << 62)
        c = rng.randrange(a + b + 1)
        trs.append((b"ABC", [a, b], [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(2)], [c, a + b - c],
                    [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(2)]))
    proofs = pp.prove_transfers_gpu(trs, seed=1)
    chk = list(range(0, n, max(1, n // 64)))
    items = [([pp.token_commit(t, v, b) for v, b in zip(iv, ib)], [pp.token_commit(t, v, b) for v, b in zip(ov, ob)],
              proofs[i]) for i, (t, iv, ib, ov, ob) in ((i, trs[i]) for i in chk)]
    st, _ = pp.verify_transfers(items)
    assert int((st != 0).sum()) == 0, "device transfer proofs rejected"
    if dist is not None:
        dist.barrier()

    class Step:
        def __init__(self, i):
            self.i, self.s = i, 0

        def verify(self):
            self.s += 1
            return pp.prove_transfers_gpu(wb, seed=1 + (self.i * 1000 + self.s) * n)

    wb = fts_gpu.WitnessBatch(trs, pp.rounds)  # packed once (host structs, reused by every call)
    elapsed, _ = _run_action_steps([Step(i) for i in range(max(1, args.action_inflight))], args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        done, cs = 0, 0.0
        while cs < args.cpu_seconds and done < n:
            c = min(thr * 32, n - done)
            t1 = time.perf_counter()
            outs = [None] * c

            def work(w):
                for j in range(w, c, thr):
                    t, iv, ib, ov, ob = trs[done + j]
                    outs[j] = pp.prove_transfer(t, iv, ib, ov, ob, seed=1 + done + j)

            ths = [threading.Thread(target=work, args=(w,)) for w in range(thr)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            cs += time.perf_counter() - t1
            assert outs == proofs[done:done + c], "host and device transfer proofs differ"
            done += c
        cpu = {"value": round(done / cs, 1), "unit": "transfer proofs/s", "cores": thr, "kind": "port",
               "sample": "%d of the same transfers, the library's host prover (fts_transfer_prove, byte-identical "
                         "output), %d threads, %.1f s wall" % (done, thr, cs)}
    if rank == 0:
        print(json.dumps({
            "metric": "2-in/2-out transfer proves/sec (TypeAndSum + 2 x rp64, BN254)", "value": round(value, 1),
            "unit": "transfer proofs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: %d seeded 2-in/2-out transfers of type ABC (seed 0xF7A500B1 + rank)" % n,
            "config": {"workload": "SURVEY 8f rank 2: %d transfers per GPU per step via fts_transfer_prove_batch_gpu, "
                                   "%d calls in flight" % (n, max(1, args.action_inflight)),
                       "transfers_per_gpu": n, "parallelism": "shard%d" % world},
            "cpu_baseline": cpu, "kernel_ms": {k: round(v[0], 4) for k, v in pp.last_timings_ex().items()}}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_audit(args):
    """the auditor's / wallet's token opening checks
    (auditor.go:226-238, token.go:69-83).  One step = one fts_token_open_batch
    over --tokens openings (host structs in: HashToZr of the type, scalar
    reduction and upload included), --action-inflight calls concurrently."""
    world, rank, local, dist = _dist_setup()
    import random
    import numpy as np
    import fts_gpu
    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=args.bits, device=local)
    t0 = time.time()
    rng = random.Random(0xF7A500A0 + rank)
    distinct = []
    for i in range(1024):
        v, bf = rng.randrange(2**64), rng.randrange(R_ORDER)
        t = b"TOK%d" % (i % 8)
        distinct.append((pp.token_commit(t, v, bf.to_bytes(32, "big")), t, v.to_bytes(32, "big"),
                         bf.to_bytes(32, "big")))
    n = args.tokens
    ops = (distinct * (n // len(distinct) + 1))[:n]
    bad = set(range(7, n, 101))  # ~1 % tampered values
    for j in bad:
        com, t, v, bf = ops[j]
        ops[j] = (com, t, (int.from_bytes(v, "big") ^ 1).to_bytes(32, "big"), bf)
    batches = [pp.prepare_openings(ops) for _ in range(max(1, args.action_inflight))]
    setup_s = time.time() - t0
    want = np.zeros(n, dtype=np.int32)
    want[sorted(bad)] = fts_gpu.FTS_E_OPEN_MISMATCH

    class Step:
        def __init__(self, b):
            self.b = b

        def verify(self):
            st = pp.check_openings(self.b)
            assert (st == want).all(), "opening verdicts differ"
            return st

    steps_objs = [Step(b) for b in batches]
    for _ in range(max(1, args.warmup)):
        steps_objs[0].verify()
    if dist is not None:
        dist.barrier()
    elapsed, _ = _run_action_steps(steps_objs, args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    # isolated kernel time (one call alone on the GPU)
    kt = {}
    reps = 4
    for _ in range(reps):
        steps_objs[0].verify()
        for name, (ms, mads) in pp.last_timings_ex().items():
            o = kt.get(name, (0.0, 0.0))
            kt[name] = (o[0] + ms, mads)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from oracle import cref, pp as oppm
        opp = oppm.load_pp(pp_raw)
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        done, cs = 0, 0.0
        while cs < args.cpu_seconds and done < n:
            c = min(2048, n - done)
            t1 = time.perf_counter()
            got = cref.open_check_many(opp, ops[done:done + c], threads=thr)
            cs += time.perf_counter() - t1
            assert got == [int(w) for w in want[done:done + c]], "CPU oracle verdicts differ"
            done += c
        cpu = {"value": round(done / cs, 1), "unit": "openings/s", "cores": thr, "kind": "port",
               "sample": "%d of the same openings, reference-order commit() (3 G1.Mul + 2 Add + Equals; "
                         "oracle/c/ref_verify.c oracle_open_check_many), %d threads, %.1f s wall" % (done, thr, cs)}
    if rank == 0:
        print(json.dumps({
            "metric": "token opening checks/sec (auditor InspectOutput, BN254)", "value": round(value, 1),
            "unit": "openings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: 1024 distinct openings (8 types) from the library's host commitment, tiled; "
                    "1 % tampered values (seed 0xF7A500A0 + rank)",
            "config": {"workload": "SURVEY 8f rank 3: %d token openings per GPU per step via fts_token_open_batch, "
                                   "%d calls in flight" % (n, len(batches)), "tokens_per_gpu": n,
                       "parallelism": "shard%d" % world},
            "roofline": _roofline_from(kt, reps), "cpu_baseline": cpu,
            "kernel_ms": {k: round(v[0] / reps, 4) for k, v in kt.items()}, "setup_s": round(setup_s, 2)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _ecdsa_muls_per_verify():
    """Montgomery products one k_ecdsa_verify lane executes per valid
    signature (csrc/ecdsa_kernels.hip; madd 11, full add 16, a=-3 dbl 8):
    pk check 5 + s^-1 by Fermat with a 4-bit window (14 table products +
    252 sqr + one product per non-zero lower nibble of n-2) + u1, u2 2 +
    u1*G 16 madd (16-bit windows) + Q table 1..8 (6 madd + 1 dbl) + 252 dbl + 60 expected adds
    (64 nibbles x 15/16) + final add 16 + projective x-compare 3."""
    n = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    nz = sum(1 for i in range(63) if ((n - 2) >> (4 * i)) & 15)
    return 5 + 1 + 14 + 252 + nz + 2 + 16 * 11 + 6 * 11 + 8 + 252 * 8 + 60 * 16 + 16 + 3


def bench_ecdsa(args):
    """SURVEY §8f rank 4 (x509 half): owner-signature checks of
    TransferSignatureValidate (validator/validator_transfer.go:29-62) ->
    ecdsa.Verifier.Verify (validator/ecdsa/ecdsa.go:82-113).  One step = one
    fts_ecdsa_verify_batch over --sigs (message, DER signature, P-256 key)
    triples from host buffers (DER parse, packing, upload, SHA-256 and the
    verification on the device, verdicts back)."""
    world, rank, local, dist = _dist_setup()
    import random
    import numpy as np
    from fts_gpu import ecdsa as E
    from oracle import ecdsa_p256 as O
    t0 = time.time()
    rng = random.Random(0xF7A5EC00 + rank)
    ndist, L = 512, args.msg_len
    keys = []
    for _ in range(16):
        d = rng.randrange(1, O.N)
        Q = O.mul(d, O.G)
        keys.append((d, Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")))
    dm, ds, dp = [], [], []
    for i in range(ndist):
        d, pk = keys[i % len(keys)]
        m = rng.randbytes(L)
        dm.append(m)
        ds.append(O.sign(d, m, rng.randrange(1, O.N)))
        dp.append(pk)
    n = args.sigs
    idx = np.arange(n) % ndist
    msg_buf = bytearray(b"".join(dm[i] for i in idx))
    bad = np.arange(13, n, 97)  # ~1 % tampered messages
    for j in bad:
        msg_buf[j * L] ^= 1
    sig_lens = np.array([len(ds[i]) for i in idx], dtype=np.uint64)
    sig_off = np.concatenate([[0], np.cumsum(sig_lens)[:-1]]).astype(np.uint64)
    sig_buf = b"".join(ds[i] for i in idx)
    pk_buf = b"".join(dp[i] for i in idx)
    msg_off = np.arange(n, dtype=np.uint64) * L
    msg_len = np.full(n, L, dtype=np.uint64)
    msg_buf = bytes(msg_buf)
    want = np.zeros(n, dtype=np.int32)
    want[bad] = E.FTS_E_SIG_INVALID
    setup_s = time.time() - t0

    def step():
        st = E.verify_packed(msg_buf, msg_off, msg_len, sig_buf, sig_off, sig_lens, pk_buf, device=local)
        assert (st == want).all(), "ECDSA verdicts differ"
        return st

    class Step:
        verify = staticmethod(step)

    for _ in range(max(1, args.warmup)):
        step()
    if dist is not None:
        dist.barrier()
    # --action-inflight concurrent calls: each runs on its own library slot
    # (stream + staging), so one call's host parse/pack overlaps another's kernels
    inflight = max(1, args.action_inflight)
    elapsed, _ = _run_action_steps([Step() for _ in range(inflight)], args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    # isolated kernel times (one call alone on the GPU), HIP events
    reps = 4
    kt = {"k_ecdsa_digest": 0.0, "k_ecdsa_verify": 0.0}
    for _ in range(reps):
        step()
        for k, v in E.last_timings(local).items():
            kt[k] += v
    steps_timed = args.steps
    muls = _ecdsa_muls_per_verify()
    mads = (n - len(bad)) * muls * MAD_PER_MUL + len(bad) * muls * MAD_PER_MUL  # tampered items run the full path
    ms = kt["k_ecdsa_verify"] / reps
    ach = mads / (ms * 1e-3) / 1e12
    roof = {"bound": "int32_valu (v_mad_u64_u32)", "kernel": "k_ecdsa_verify", "achieved": round(ach, 3),
            "peak": round(PEAK_TMAD, 3), "unit": "TMAD/s", "frac": round(ach / PEAK_TMAD, 4), "traffic": None,
            "kernel_ms": round(ms, 4), "mads_per_launch": mads, "muls_per_verify": muls,
            "measured": "HIP events around each launch on the library's stream, %d isolated calls after the "
                        "timed region" % reps}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        done, t2 = 0, time.perf_counter()
        while time.perf_counter() - t2 < min(args.cpu_seconds, 10.0) and done < n:
            i = int(idx[done])
            m = msg_buf[done * L:(done + 1) * L]
            got = O.verify(m, ds[i], (int.from_bytes(dp[i][:32], "big"), int.from_bytes(dp[i][32:], "big")))
            assert got == want[done], "CPU oracle verdict differs"
            done += 1
        cs = time.perf_counter() - t2
        cpu = {"value": round(done / cs, 1), "unit": "signatures/s", "cores": 1, "kind": "port",
               "sample": "first %d signatures of the batch, oracle/ecdsa_p256.py (pure-Python restatement of "
                         "Verifier.Verify, affine double-and-add), 1 thread, %.1f s wall" % (done, cs)}
    if rank == 0:
        print(json.dumps({
            "metric": "ECDSA P-256 owner signature verifies/sec (Verifier.Verify)", "value": round(value, 1),
            "unit": "signatures/s", "n_gpus": world, "steps": steps_timed, "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps_timed * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (P-256 Fp/Fn 8x32-bit Montgomery)",
            "data": "synthetic: %d distinct signatures (16 keys, %d-byte messages) from the oracle signer, tiled; "
                    "1 %% tampered messages (seed 0xF7A5EC00 + rank)" % (ndist, L),
            "config": {"workload": "SURVEY 8f rank 4 (x509): %d owner signatures per GPU per step via "
                                   "fts_ecdsa_verify_batch, %d calls in flight" % (n, inflight), "sigs_per_gpu": n, "msg_len": L,
                       "parallelism": "shard%d" % world},
            "roofline": roof, "cpu_baseline": cpu,
            "kernel_ms": {k: round(v / reps, 4) for k, v in kt.items()}, "setup_s": round(setup_s, 2)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


# products of one nym verification (k_nym_verify): HSk and HRand fixed-base products
# (16-bit windows: 15 mixed additions of 11 products after the first copy), the GLV
# product c*Nym (straus2_128: 2 x (1 dbl + 6 adds) table, 124 doublings of 7, ~60
# additions of 16), the on-curve check (4); SHA-256 and the inversion are not counted
NYM_MULS_PER_VERIFY = 2 * 15 * 11 + 2 * (7 + 6 * 16) + 124 * 7 + 60 * 16 + 4


def bench_idemix(args):
    """SURVEY §8f rank 4 (idemix half): owner-signature checks of
    TransferSignatureValidate (validator/validator_transfer.go:29-62) for
    idemix-owned inputs -> crypto.NymSignatureVerifier.Verify
    (services/identity/idemix/crypto/id.go:145-161).  One step = one
    fts_nym_verify_batch over --sigs (nym key, NymSignature, message) triples
    from host buffers under the BN254 issuer key of zkatdlog_pp.json
    (proto parse, packing, upload, the curve work and both hashes on the
    device, verdicts back)."""
    world, rank, local, dist = _dist_setup()
    import random
    import numpy as np
    from fts_gpu import idemix as I
    from oracle import idemix as O
    t0 = time.time()
    bn = args.idemix_curve == "bn254"
    C = O.BN254C if bn else O.FP256BNC
    kdir = "bn254_tokengen" if bn else "fp256bn_validator"
    with open(os.path.join(ROOT, "tests", "golden", "idemix", kdir, "IssuerPublicKey"), "rb") as f:
        ipk_raw = f.read()
    ipk = O.parse_ipk(ipk_raw, C)
    rng = random.Random(0xF7A51D00 + rank)
    ndist, L = 256, args.msg_len
    keys = []
    for _ in range(16):
        sk, rn = rng.randrange(C.r), rng.randrange(C.r)
        keys.append((sk, rn, O.make_nym(ipk, sk, rn)))
    dn, ds, dm = [], [], []
    for i in range(ndist):
        sk, rn, nym = keys[i % len(keys)]
        m = rng.randbytes(L)
        dm.append(m)
        ds.append(O.nym_sign(ipk, sk, nym, rn, m, rng))
        dn.append(C.g1_bytes(nym))
    n = args.sigs
    idx = np.arange(n) % ndist
    msg_buf = bytearray(b"".join(dm[i] for i in idx))
    bad = np.arange(13, n, 97)  # ~1 % tampered messages
    for j in bad:
        msg_buf[j * L] ^= 1
    msg_buf = bytes(msg_buf)
    sig_lens = np.array([len(ds[i]) for i in idx], dtype=np.uint64)
    sig_off = np.concatenate([[0], np.cumsum(sig_lens)[:-1]]).astype(np.uint64)
    sig_buf = b"".join(ds[i] for i in idx)
    nym_buf = b"".join(dn[i] for i in idx)
    msg_off = np.arange(n, dtype=np.uint64) * L
    msg_len = np.full(n, L, dtype=np.uint64)
    want = np.zeros(n, dtype=np.int32)
    want[bad] = I.FTS_E_NYM_INVALID
    K = I.IssuerKey(ipk_raw, device=local, curve=I.FTS_CURVE_BN254 if bn else I.FTS_CURVE_FP256BN_AMCL)
    setup_s = time.time() - t0

    def step():
        st = K.verify_packed(nym_buf, sig_buf, sig_off, sig_lens, msg_buf, msg_off, msg_len)
        assert (st == want).all(), "idemix verdicts differ"
        return st

    class Step:
        verify = staticmethod(step)

    for _ in range(max(1, args.warmup)):
        step()
    if dist is not None:
        dist.barrier()
    inflight = max(1, args.action_inflight)
    elapsed, _ = _run_action_steps([Step() for _ in range(inflight)], args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    reps, kms = 4, 0.0
    for _ in range(reps):
        step()
        kms += K.last_kernel_ms()
    ms = kms / reps
    # FP256BN: 2 x 16 mixed additions, GLV tables 2 x 7 mixed additions, 128 doublings,
    # <= 2 x 33 full additions (~64), beta and the on-curve check (5)
    muls = NYM_MULS_PER_VERIFY if bn else 2 * 16 * 11 + 14 * 11 + 128 * 7 + 64 * 16 + 5
    mads = n * muls * MAD_PER_MUL  # tampered items run the full path
    ach = mads / (ms * 1e-3) / 1e12
    roof = {"bound": "int32_valu (v_mad_u64_u32)", "kernel": "k_nym_verify" + ("" if bn else "_fbn"), "achieved": round(ach, 3),
            "peak": round(PEAK_TMAD, 3), "unit": "TMAD/s", "frac": round(ach / PEAK_TMAD, 4), "traffic": None,
            "kernel_ms": round(ms, 4), "mads_per_launch": mads, "muls_per_verify": muls,
            "measured": "HIP events around each launch on the library's stream, %d isolated calls after the "
                        "timed region (SHA-256 and the inversion not counted as work)" % reps}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        done, t2 = 0, time.perf_counter()
        while time.perf_counter() - t2 < min(args.cpu_seconds, 10.0) and done < n:
            i = int(idx[done])
            m = msg_buf[done * L:(done + 1) * L]
            try:
                O.nym_verify(ipk, dn[i], ds[i], m)
                got = 0
            except O.NymError:
                got = I.FTS_E_NYM_INVALID
            assert got == want[done], "CPU oracle verdict differs"
            done += 1
        cs = time.perf_counter() - t2
        cpu = {"value": round(done / cs, 1), "unit": "signatures/s", "cores": 1, "kind": "port",
               "sample": "first %d signatures of the batch, oracle/idemix.py (pure-Python restatement of "
                         "NymSignature.Ver, affine double-and-add), 1 thread, %.1f s wall" % (done, cs)}
    K.close()
    if rank == 0:
        print(json.dumps({
            "metric": "idemix nym signature verifies/sec (NymSignatureVerifier.Verify, %s)" % C.name,
            "value": round(value, 1), "unit": "signatures/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (%s Fp/Fr 8x32-bit Montgomery)" % C.name,
            "data": "synthetic: %d distinct nym signatures (16 nyms, %d-byte messages) from the oracle signer under "
                    "the %s issuer key (%s), tiled; 1 %% tampered messages (seed 0xF7A51D00 + rank)"
                    % (ndist, L, C.name, kdir),
            "config": {"workload": "SURVEY 8f rank 4 (idemix): %d owner signatures per GPU per step via "
                                   "fts_nym_verify_batch, %d calls in flight" % (n, inflight), "sigs_per_gpu": n,
                       "msg_len": L, "parallelism": "shard%d" % world},
            "roofline": roof, "cpu_baseline": cpu, "kernel_ms": {"k_nym_verify" + ("" if bn else "_fbn"): round(ms, 4)},
            "setup_s": round(setup_s, 2)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# Fp products of one identity check (cost model of csrc/idemix_identity.hip, BN254 loop
# lengths): Fp2 mul 3, Fp6 mul 18, Fp12 mul 54 / sqr 36, sparse line product 44.
#   pairing: multi-Miller loop of 2 pairings over |6u+2| (65 bits, 37 set): 63 squarings,
#   (64 + 36 + 2) x 2 line products; final exponentiation: easy part ~250, hard part 3
#   exponentiations by u (62 cyclotomic squarings of 18 + 27 products each) + ~10 products,
#   4 cyclotomic squarings, 8 Frobenius
#   t-values: 6 GLV products (table 103 + normalisation 53 + 124 doublings of 7 + ~60 mixed
#   additions of 11 + ~30 beta products) + 11 distinct fixed-base products (16 mixed additions;
#   round 6: three of the reference's 14 repeat with the same base and scalar) + 20 additions
ID_PAIRING_MULS = 63 * 36 + (64 + 36 + 2) * 2 * 44 + 250 + 3 * (62 * 18 + 27 * 54) + 10 * 54 + 4 * 18 + 8 * 15
ID_TVAL_MULS = 6 * (103 + 53 + 124 * 7 + 60 * 11 + 30) + 11 * 16 * 11 + 20 * 16 + 65
#   batch pairing check: two 64-bit GLV chains (table 103 + normalisation 53 + 64 doublings
#   of 7 + ~32 mixed additions of 11 + ~16 beta products) and one LDS-tree addition of 16 each
ID_BATCH_MULS = 2 * (103 + 53 + 64 * 7 + 32 * 11 + 16 + 16)


def bench_identity(args):
    """SURVEY §8f rank 4 (idemix half): identity validity of idemix owners, checked
    for every transfer input by GetOwnerVerifier -> Deserializer.Deserialize(raw, true)
    (validator/validator_transfer.go:46, services/identity/idemix/deserializer.go:83,
    crypto/id.go:74-108: IBM/idemix Signature.Ver).  One step = one
    fts_idemix_identity_verify_batch over --sigs serialized identities (host proto
    parse, upload, decode + t-values + transcript kernel, pairing kernel, verdicts back)."""
    world, rank, local, dist = _dist_setup()
    import numpy as np
    from fts_gpu import idemix as I
    t0 = time.time()
    tag = args.idemix_curve
    with open(os.path.join(ROOT, "tests", "golden", "idemix_identity_golden.json")) as f:
        doc = json.load(f)[tag]
    with open(os.path.join(ROOT, "tests", "golden", "idemix", doc["issuer"], "IssuerPublicKey"), "rb") as f:
        ipk_raw = f.read()
    pool = [(bytes.fromhex(t["identity"]), t["error"]) for t in doc["tile"]]  # 64 identities, 1 in 8 tampered
    n = args.sigs
    order = (np.arange(n) * 7 + 13 * rank) % len(pool)
    ids = [pool[k][0] for k in order]
    want_ok = np.array([pool[k][1] is None for k in order])
    V = I.IdentityVerifier(ipk_raw, device=local, curve=doc["curve_id"])
    setup_s = time.time() - t0

    prep = V.prepare(ids)  # the C-ABI's pointer arrays, built once (as a Go caller passes its slices)

    def step():
        st = V.verify_prepared(prep)
        assert ((st == 0) == want_ok).all(), "identity verdicts differ"
        return st

    class Step:
        verify = staticmethod(step)

    for _ in range(max(1, args.warmup)):
        step()
    if dist is not None:
        dist.barrier()
    inflight = max(1, args.action_inflight)
    elapsed, _ = _run_action_steps([Step() for _ in range(inflight)], args.steps, None, None)
    elapsed = _max_over_ranks(dist, elapsed)
    value = world * n * args.steps / elapsed
    reps, kt, kp = 4, 0.0, 0.0
    for _ in range(reps):
        step()
        a, b = V.last_kernel_ms()
        kt, kp = kt + a, kp + b
    kt, kp = kt / reps, kp / reps
    groups, paired = V.last_pairing_stats()
    # the dominant device work since the batch pairing check (round 6): the t-value
    # kernels (k_idv_var's six GLV and eleven fixed-base products per identity); the
    # pairing phase is mostly the latency of the per-group pairings (a few waves)
    mads = n * ID_TVAL_MULS * MAD_PER_MUL
    ach = mads / (kt * 1e-3) / 1e12
    # HBM bytes of the three t-value launches at 65,536 identities (BN254), from the newest
    # profiles/identity_traffic_rNN.json (separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes)
    traffic, tsrc = None, None
    if tag == "bn254" and n == 65536:
        import glob
        cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "identity_traffic_r[0-9][0-9].json")))
        try:
            tj = json.load(open(cands[-1]))
            traffic = sum(int(tj[k]["fetch_bytes_raw"]) + int(tj[k]["write_bytes"])
                          for k in ("k_idv_decode", "k_idv_var", "k_idv_tvals"))
            tsrc = os.path.basename(cands[-1])
        except (IndexError, OSError, KeyError, ValueError):
            traffic = None
    roof = {"bound": "int32_valu (v_mad_u64_u32)", "kernel": "k_idv_decode + k_idv_var + k_idv_tvals",
            "achieved": round(ach, 3), "peak": round(PEAK_TMAD, 3), "unit": "TMAD/s", "frac": round(ach / PEAK_TMAD, 4),
            "traffic": traffic, "traffic_source": tsrc, "kernel_ms": round(kt, 4), "mads_per_launch": mads,
            "muls_per_identity": ID_TVAL_MULS,
            "measured": "HIP events around the three launches on the library's stream, %d isolated calls after the "
                        "timed region (the Fp inversions are not counted as work)" % reps}
    pairing = {"phase_ms": round(kp, 4), "groups": groups, "paired_one_by_one": paired,
               "batch_muls_per_identity": ID_BATCH_MULS,
               "note": "k_idv_bp_terms (two 64-bit GLV chains per identity), one randomised pairing product per "
                       "group of 256 (k_idv_bp_pair), one-by-one pairings only for failing groups; "
                       "FTS_IDV_BATCH=0 pairs every identity (%d Fp products each)" % ID_PAIRING_MULS}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from oracle import idemix as O, idemix_identity as ID, pairing as PR
        C, PC = (O.BN254C, PR.BN254) if tag == "bn254" else (O.FP256BNC, PR.FP256BN)
        ipk = O.parse_ipk(ipk_raw, C)
        W = ID.ipk_w(PC, ipk_raw)
        done, t2 = 0, time.perf_counter()
        while time.perf_counter() - t2 < min(args.cpu_seconds, 10.0) and done < n:
            try:
                ID.verify_identity(ipk, PC, W, ids[done])
                ok = True
            except ID.IdentityError:
                ok = False
            assert ok == want_ok[done], "CPU oracle verdict differs"
            done += 1
        cs = time.perf_counter() - t2
        cpu = {"value": round(done / cs, 3), "unit": "identities/s", "cores": 1, "kind": "port",
               "sample": "first %d identities of the batch, oracle/idemix_identity.py (pure-Python restatement of "
                         "Signature.Ver with a direct E(Fp12) pairing), 1 thread, %.1f s wall" % (done, cs)}
    V.close()
    if rank == 0:
        print(json.dumps({
            "metric": "idemix identity validity checks/sec (Deserialize(raw, true) -> Signature.Ver, %s)" % tag,
            "value": round(value, 1), "unit": "identities/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (%s Fp 8x32-bit Montgomery, Fp12 tower)" % tag,
            "data": "the 64 oracle-made identities of tests/golden/idemix_identity_golden.json (from the reference's "
                    "%s SignerConfig credential; 1 in 8 with a tampered response), tiled" % doc["issuer"],
            "config": {"workload": "SURVEY 8f rank 4 (idemix identity): %d identities per GPU per step via "
                                   "fts_idemix_identity_verify_batch, %d calls in flight" % (n, inflight),
                       "identities_per_gpu": n, "parallelism": "shard%d" % world},
            "roofline": roof, "cpu_baseline": cpu,
            "kernel_ms": {"k_idv_tvals": round(kt, 4), "k_idv_pairing": round(kp, 4)}, "pairing_check": pairing,
            "tval_mads_per_identity": ID_TVAL_MULS * MAD_PER_MUL, "setup_s": round(setup_s, 2)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_transfer(args, raw_requests=False):
    """C4: 2-in/2-out transfers.  raw_requests: the same transfers, each wrapped in
    its own serialized TokenRequest (1 transfer action, signatures attached) and
    verified through fts_request_verify_batch -- protobuf decode, structural checks
    and G1 JSON decoding included in the timed region"""
    world, rank, local, dist = _dist_setup()
    import random
    import numpy as np
    import fts_gpu
    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=args.bits, device=local)
    T = b"ABC"
    rng = random.Random(0xF7A50004 + rank)
    t0 = time.time()
    distinct = min(args.transfers, 512)
    base = []
    for i in range(distinct):
        a, b_ = rng.getrandbits(args.bits - 2), rng.getrandbits(args.bits - 2)
        c = rng.randrange(a + b_ + 1)
        inv, outv = [a, b_], [c, a + b_ - c]
        ib = [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(2)]
        ob = [rng.randrange(R_ORDER).to_bytes(32, "big") for _ in range(2)]
        ins = [pp.token_commit(T, v, bf) for v, bf in zip(inv, ib)]
        outs = [pp.token_commit(T, v, bf) for v, bf in zip(outv, ob)]
        base.append((ins, outs, pp.prove_transfer(T, inv, ib, outv, ob, 0xF7A50004 + i)))
    items = [base[i % distinct] for i in range(args.transfers)]
    nb = max(1, min(args.action_inflight, args.steps))
    if raw_requests:
        R = fts_gpu.request
        reqs = []
        for i, (ins, outs, proof) in enumerate(items):
            ta = R.transfer_action([("%064x" % (i * 2 + k), k, b"owner-%d" % i, c) for k, c in enumerate(ins)],
                                   [(b"recipient-%d" % i, c) for c in outs], proof)
            reqs.append(R.token_request([(R.TRANSFER, ta)], [b"\x30" * 72, b"\x30" * 72]))
        batches = [pp.prepare_requests(reqs) for _ in range(nb)]
    else:
        batches = [pp.prepare_transfers(items) for _ in range(nb)]
    pp.reserve()  # every lane's workspace sized for the largest pass, before the clock (as C2)
    setup_s = time.time() - t0
    for _ in range(max(1, args.warmup)):
        st, fi = batches[0].verify()[0], None
    assert int((st != 0).sum()) == 0, "honest transfers rejected"
    _run_action_steps(batches, nb, None, None)
    if dist is not None:
        dist.barrier()
    from fts_gpu import dist as fdist
    # host buffers in (the C-ABI parses the DER proofs), verdicts out
    elapsed, _ = _run_action_steps(batches, args.steps, dist, lambda r: fdist.allgather_verdicts(dist, r[0]))
    elapsed = _max_over_ranks(dist, elapsed)
    kt = {k: (v[0] * args.steps, v[1]) for k, v in pp.last_timings_ex().items()}
    value = world * args.transfers * args.steps / elapsed
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0 and not raw_requests:
        acts = [("transfer", ins, outs, proof) for ins, outs, proof in items]
        cpu = _action_cpu_baseline(pp_raw, args.bits, acts, [(0, -1)] * len(acts), args, "transfer verifies/s",
                                   "2-in/2-out %d-bit transfers" % args.bits)
    if raw_requests:
        metric = "raw TokenRequest verifies/sec (1 transfer 2-in/2-out each, BN254, %d-bit range proofs)" % args.bits
        unit, entry = "requests/s", "fts_request_verify_batch (protobuf + G1 JSON decode in the timed region)"
    else:
        metric = "2-in/2-out transfer verifies/sec (BN254, %d-bit range proofs)" % args.bits
        unit, entry = "transfers/s", "fts_transfer_verify_batch"
    if rank == 0:
        print(json.dumps({
            "metric": metric,
            "value": round(value, 1), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: %d distinct 2-in/2-out transfers (type ABC) from the library's host prover, tiled"
                    % distinct,
            "config": {"workload": "C4 per GPU: %d transfers (TypeAndSum + 2 rp%d each) per step via "
                                   "%s, %d calls in flight" % (args.transfers, args.bits, entry, nb),
                       "transfers_per_gpu": args.transfers, "parallelism": "shard%d" % world},
            "roofline": _msm_roofline(kt, args), "cpu_baseline": cpu,
            "kernel_ms": {k: round(v[0] / args.steps, 4) for k, v in kt.items()}, "setup_s": round(setup_s, 2)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_mixed(args):
    """C5: issue(16 outputs) : transfer(2-in/2-out) = 1 : 4 at 32-bit range,
    1 % of the actions tampered (wrong committed value), one pass per step"""
    world, rank, local, dist = _dist_setup()
    import random
    import numpy as np
    import fts_gpu
    bits = 32
    with open(os.path.join(ROOT, "tests", "golden", "zkatdlog_pp.json"), "rb") as f:
        pp_raw = f.read()
    pp = fts_gpu.PublicParams(pp_raw, bit_length=bits, device=local)
    T = b"ABC"
    rng = random.Random(0xF7A50005 + rank)
    n_tr = args.transfers
    n_is = n_tr // 4
    t0 = time.time()

    def bf():
        return rng.randrange(R_ORDER).to_bytes(32, "big")

    def transfer(bad):
        a, b_ = rng.getrandbits(bits - 2), rng.getrandbits(bits - 2)
        c = rng.randrange(a + b_ + 1)
        inv, outv = [a, b_], [c, a + b_ - c]
        ib, ob = [bf(), bf()], [bf(), bf()]
        ins = [pp.token_commit(T, v, x) for v, x in zip(inv, ib)]
        outs = [pp.token_commit(T, v + (1 if bad and j == 0 else 0), x) for j, (v, x) in enumerate(zip(outv, ob))]
        return ins, outs, pp.prove_transfer(T, inv, ib, outv, ob, rng.getrandbits(63))

    def issue(bad):
        vals = [rng.getrandbits(bits) for _ in range(16)]
        bfs = [bf() for _ in range(16)]
        toks = [pp.token_commit(T, v, x) for v, x in zip(vals, bfs)]
        if bad:
            toks[rng.randrange(16)] = pp.token_commit(T, vals[0] ^ 1, bfs[0])
        return toks, pp.prove_issue(T, vals, bfs, rng.getrandbits(63))

    dt, di = min(n_tr, 256), min(n_is, 64)
    tr_base = [transfer(False) for _ in range(dt)]
    is_base = [issue(False) for _ in range(di)]
    bad_tr = set(rng.sample(range(n_tr), max(1, n_tr // 100)))
    bad_is = set(rng.sample(range(n_is), max(1, n_is // 100)))
    tr_bad = {i: transfer(True) for i in bad_tr}
    is_bad = {i: issue(True) for i in bad_is}
    transfers = [tr_bad.get(i, tr_base[i % dt]) for i in range(n_tr)]
    issues = [is_bad.get(i, is_base[i % di]) for i in range(n_is)]
    nb = max(1, min(args.action_inflight, args.steps))
    batches = [pp.prepare_actions(transfers, issues) for _ in range(nb)]
    pp.reserve()  # every lane's workspace sized for the largest pass, before the clock (as C2)
    setup_s = time.time() - t0
    for _ in range(max(1, args.warmup)):
        st_t, fi_t, st_i, fi_i = batches[0].verify()
    assert set(np.nonzero(st_t)[0]) == bad_tr and set(np.nonzero(st_i)[0]) == bad_is, "verdict mismatch"
    _run_action_steps(batches, nb, None, None)
    if dist is not None:
        dist.barrier()
    from fts_gpu import dist as fdist
    elapsed, outs = _run_action_steps(batches, args.steps, dist,
                                      lambda r: fdist.allgather_verdicts(dist, np.concatenate([r[0], r[2]])))
    elapsed = _max_over_ranks(dist, elapsed)
    for o in outs:
        for r in o:
            assert set(np.nonzero(r[0])[0]) == bad_tr and set(np.nonzero(r[2])[0]) == bad_is
    kt = {k: (v[0] * args.steps, v[1]) for k, v in pp.last_timings_ex().items()}
    value = world * (n_tr + n_is) * args.steps / elapsed
    # one call alone after the timed region: the fallback's own cost (in the
    # pipelined region the latency-bound fallback kernels share the CUs with the
    # other calls' passes, which stretches their spans)
    iso_reps = 3
    kti, t_iso = {}, time.perf_counter()
    for _ in range(iso_reps):
        batches[0].verify()
        for kname, (ms, mads) in pp.last_timings_ex().items():
            o = kti.get(kname, (0.0, 0.0))
            kti[kname] = (o[0] + ms, mads)
    iso_ms = (time.perf_counter() - t_iso) * 1e3 / iso_reps
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        # the same interleaving as the batch (1 issue : 4 transfers), verdicts from the GPU run
        order = []
        for j in range(n_is):
            order += [("t", 4 * j + q) for q in range(4) if 4 * j + q < n_tr] + [("i", j)]
        acts, want = [], []
        for kind, i in order:
            if kind == "t":
                ins, outs, proof = transfers[i]
                acts.append(("transfer", ins, outs, proof))
                want.append((int(st_t[i]), int(fi_t[i])))
            else:
                toks, proof = issues[i]
                acts.append(("issue", [], toks, proof))
                want.append((int(st_i[i]), int(fi_i[i])))
        cpu = _action_cpu_baseline(pp_raw, bits, acts, want, args, "actions/s",
                                   "mixed actions (1 issue-16 : 4 transfers, 32-bit)")
    if rank == 0:
        print(json.dumps({
            "metric": "mixed action verifies/sec (issue-16 + 2-in/2-out transfers, BN254, 32-bit)",
            "value": round(value, 1), "unit": "actions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (BN254 Fp/Fr 8x32-bit Montgomery)",
            "data": "synthetic: %d transfers + %d issues (16 outputs) per GPU, 1 %% tampered, host prover" % (n_tr, n_is),
            "config": {"workload": "C5 per GPU: 1 issue-16 : 4 transfers at 32-bit, one fts_actions_verify_batch "
                                   "per step (%d range proofs), %d calls in flight" % (2 * n_tr + 16 * n_is, nb),
                       "transfers_per_gpu": n_tr, "issues_per_gpu": n_is, "parallelism": "shard%d" % world},
            "roofline": _roofline_from(kt, args.steps), "cpu_baseline": cpu,
            "fallback": _fallback_share(kti, iso_reps, iso_ms),
            "fallback_pipelined": _fallback_share(kt, args.steps, elapsed / args.steps * nb * 1e3),
            "isolated_call_ms": round(iso_ms, 3),
            "kernel_ms_isolated": {k: round(v[0] / iso_reps, 4) for k, v in kti.items()},
            "kernel_ms": {k: round(v[0] / args.steps, 4) for k, v in kt.items()}, "setup_s": round(setup_s, 2)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _tamper_note(args, B):
    if args.tamper <= 0:
        return ""
    if args.tamper_every > 1:
        return ", %d tampered proof(s) in every %d-th batch" % (max(1, round(args.tamper * B)), args.tamper_every)
    return ", %g %% tampered" % (100 * args.tamper)


def _fallback_share(kt, steps, call_ms):
    """device time of the batch check's fallback (group test + per-proof checks,
    "fb:" kernels) per call, against all kernel time and against the call's wall
    time (ms_per_step x calls in flight)"""
    fb = sum(v[0] for k, v in kt.items() if k.startswith("fb:")) / steps
    dev = sum(v[0] for k, v in kt.items() if not k.startswith("host_")) / steps
    return {"kernel_ms_per_call": round(fb, 3), "share_of_kernel_time": round(fb / dev, 4) if dev else None,
            "call_wall_ms": round(call_ms, 3), "share_of_call_wall": round(fb / call_ms, 4) if call_ms else None}


if __name__ == "__main__":
    main()
