"""GPU: every library knob (FTS_* environment variable read at context creation,
fts_api.cpp ctx_create) at a non-default value gives the reference's verdicts
(rp/rangecorrectness.go:141-160) and, where the knob changes the com / x0 code
path, the same exact intermediates (com, H'_i, x0: ipa.go:200-213).

Knobs covered elsewhere: FTS_LANES, FTS_COM_FIXED_MAX (test_gpu_rp.py,
test_gpu_scale.py), FTS_GT1 / FTS_GT2_MIN / FTS_GT_ADAPT (test_gpu_scale.py),
FTS_NYM_TILE (test_idemix.py), FTS_MAIN_GROUPS (test_gpu_scale.py).  Here:
FTS_RLC_FORK, FTS_X0_SPLIT, FTS_COALESCE_MAX, FTS_GATHER_US, FTS_GT_ADAPT=0,
FTS_MSM_SORT, FTS_WIDE_BITS, FTS_WAVE_PRIO, FTS_WORK_BS, FTS_GATHER_TARGET,
FTS_FX_SERIAL, FTS_MSM_MAXC.  FTS_IDLE_GATHER_US /
FTS_IDLE_QUIET_US: test_gpu_scale.py (the idle-burst split and the blocker tests)."""
import json
import os
import random
import threading

import numpy as np
import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, zkat

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "rp_golden.json")) as f:
    RP_GOLDEN = json.load(f)
STATUS_OF = {None: 0, "invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
             "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}


def _ctx(pp_raw, bits, **env):
    import fts_gpu
    env = {k: str(v) for k, v in env.items()}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fts_gpu.PublicParams(pp_raw, bit_length=bits, device=0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _golden_check(pp, bits, work_path):
    from test_gpu_rp import _intermediates
    cases = [c for c in RP_GOLDEN if c["bits"] == bits]
    st = pp.verify_range_proofs([bytes.fromhex(c["proof"]) for c in cases],
                                [bytes.fromhex(c["commitment"]) for c in cases])
    assert [int(s) for s in st] == [STATUS_OF[c["expect"]] for c in cases]
    lt = pp.last_timings()
    assert ("k_rp_com_var" in lt) == work_path and ("k_rp_fixed_all" in lt) == (not work_path), sorted(lt)
    for i, c in enumerate(cases):
        vals, com, hp = _intermediates(pp, i)
        if "com" in c:
            assert com.hex() == c["com"] and [h.hex() for h in hp] == c["hprime"] and vals[7] == int(c["x0"])


@pytest.mark.parametrize("fork", [0, 1, 3, 4])
@pytest.mark.parametrize("work_path", [False, True])
def test_knob_rlc_fork(pp_raw, fork, work_path):
    """FTS_RLC_FORK=0/1/3/4 (default 2 = adaptive): the batch check forks after the
    challenges or after the fixed-base products, or (work path) sorts its MSM
    beside (3) or ahead of (4) the fixed-base launch and accumulates after it;
    on both com paths"""
    env = dict(FTS_RLC_FORK=fork, FTS_LANES=1)
    if work_path:
        env["FTS_COM_FIXED_MAX"] = 0
    pp = _ctx(pp_raw, 32, **env)
    try:
        _golden_check(pp, 32, work_path)
    finally:
        pp.close()


@pytest.mark.parametrize("work_path", [False, True])
def test_knob_x0_split_off(pp_raw, work_path):
    """FTS_X0_SPLIT=0: both com paths hash the whole x0 message after com (no
    prefix midstate on the side stream) -- the same x0 bytes"""
    env = dict(FTS_X0_SPLIT=0, FTS_LANES=1)
    if work_path:
        env["FTS_COM_FIXED_MAX"] = 0
    pp = _ctx(pp_raw, 32, **env)
    try:
        _golden_check(pp, 32, work_path)
        assert "k_rp_x0_prefix" not in pp.last_timings()
    finally:
        pp.close()


@pytest.mark.parametrize("bits", [32, 64])
def test_knob_x0_split_latency_path(pp_raw, bits):
    """FTS_X0_SPLIT=3 (default since round 6): the latency path too hashes the x0 prefix (H' records written
    by the normalisation, k_rp_x0_hdr) on the side stream beside com_tree, then the
    suffix after com -- the same verdicts, com, H' and x0"""
    pp = _ctx(pp_raw, bits, FTS_X0_SPLIT=3, FTS_LANES=1)
    try:
        _golden_check(pp, bits, False)
        assert "k_rp_x0_prefix" in pp.last_timings()
    finally:
        pp.close()


def _tampered_batches(pp, nb, per, seed):
    rng = random.Random(seed)
    R = bn.R
    vals = [rng.getrandbits(32) for _ in range(per)]
    bfs = [rng.randrange(R).to_bytes(32, "big") for _ in range(per)]
    proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=seed)
    out = []
    for b in range(nb):
        ps, want = list(proofs), np.zeros(per, dtype=np.int32)
        for q, i in enumerate(rng.sample(range(per), 3)):
            t = zkat.RangeProof.deserialize(ps[i])
            if q == 0:
                t.data.T1 = bn.g1_add(t.data.T1, bn.GEN)
                want[i] = 3
            else:
                t.ipa.L[q] = bn.g1_add(t.ipa.L[q], bn.GEN)
                want[i] = 6
            ps[i] = t.serialize()
        out.append((pp.stage_range_proofs(ps, coms), want))
    return out


@pytest.mark.parametrize("env", [
    dict(FTS_COALESCE_MAX=4096, FTS_GATHER_US=3000),   # small coalescing cap, long gather window
    dict(FTS_GATHER_US=0),                             # no gather window
    dict(FTS_GATHER_TARGET=1024, FTS_IDLE_GATHER_US=2000),  # idle burst cut at 2 batches a pass
    dict(FTS_FX_SERIAL=1),                             # one fixed-base launch at a time across lanes
], ids=["coalesce4096", "gather0", "target1024", "fx_serial"])
def test_knob_coalescing(pp_raw, env):
    """8 staged batches of 512 rp32 (3 tampered each) verified concurrently from 8
    threads: however the dispatcher groups them (coalesced passes up to the cap,
    lone passes), every batch gets its own exact verdicts"""
    pp = _ctx(pp_raw, 32, FTS_LANES=4, FTS_COM_FIXED_MAX=0, **env)
    try:
        batches = _tampered_batches(pp, 8, 512, 0xC0A1)
        for rep in range(3):
            res = [None] * len(batches)
            gate = threading.Barrier(len(batches))

            def run(j):
                gate.wait()
                res[j] = (batches[j][0].verify(), batches[j][0].merged())
            th = [threading.Thread(target=run, args=(j,)) for j in range(len(batches))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            for (st, merged), (_, want) in zip(res, batches):
                assert (st == want).all(), (rep, np.nonzero(st != want)[0][:8], merged)
        for b, _ in batches:
            b.close()
    finally:
        pp.close()


def test_knob_gt_adapt_off(pp_raw):
    """FTS_GT_ADAPT=0: a caller batch whose bad proofs are dense (every 32nd of
    512 tampered) keeps starting its group test at 256-groups on every call
    (with the default it moves to groups of 8 after the first, test_gpu_scale.py);
    the verdicts are the same on every call"""
    from test_gpu_scale import _raw_timing_names
    pp = _ctx(pp_raw, 16, FTS_GT_ADAPT=0, FTS_LANES=1)
    try:
        rng = random.Random(0x6AD0)
        m = 512
        vals = [rng.getrandbits(16) for _ in range(m)]
        bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(m)]
        proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=0x6AD0)
        want = np.zeros(m, dtype=np.int32)
        for i in range(5, m, 32):
            t = zkat.RangeProof.deserialize(proofs[i])
            if (i // 32) % 2:
                t.data.T1 = bn.g1_add(t.data.T1, bn.GEN)
                want[i] = 3
            else:
                t.ipa.R[1] = bn.g1_add(t.ipa.R[1], bn.GEN)
                want[i] = 6
            proofs[i] = t.serialize()
        b = pp.stage_range_proofs(proofs, coms)
        for rep in range(3):
            st = b.verify()
            assert (st == want).all(), (rep, np.nonzero(st != want)[0][:8])
            names, _ = _raw_timing_names(b)
            assert "fb:k_rlc_group_columns" in names, (rep, names)
        b.close()
    finally:
        pp.close()


@pytest.mark.parametrize("sort", [0, 1])
def test_knob_msm_sort(pp_raw, sort):
    """FTS_MSM_SORT=0 forces the round-4 sort of the batch check's MSM (k_msm_digits'
    device atomics + k_msm_scatter); 1 (default) the two-level counting sort
    (k_rs_*).  A 768-proof rp32 pass (11,520 MSM points: the two-level sort's range)
    with tampered proofs in it: the same exact verdicts either way, and the
    timeline names the sort that ran"""
    pp = _ctx(pp_raw, 32, FTS_MSM_SORT=sort, FTS_LANES=1, FTS_COM_FIXED_MAX=0)
    try:
        (b, want), = _tampered_batches(pp, 1, 768, 0x50A7 + sort)
        got = b.verify(want_status=True)
        assert (got == want).all(), np.nonzero(got != want)
        names = set(b.timings())
        if sort:
            assert "k_rs_part" in names and "k_msm_digits" not in names, sorted(names)
        else:
            assert "k_msm_digits" in names and "k_rs_part" not in names, sorted(names)
        # an honest batch closes the combination with either sort (no fallback)
        vals = list(range(1, 769))
        proofs, coms = pp.prove_range_batch_gpu(vals, [(7).to_bytes(32, "big")] * 768, seed=0x50A8)
        st = pp.verify_range_proofs(proofs, coms)
        assert not any(int(s) for s in st)
        assert not any(k.startswith("fb:") for k in pp.last_timings()), sorted(pp.last_timings())
        b.close()
    finally:
        pp.close()


@pytest.mark.parametrize("wbits", [20, 22])
@pytest.mark.parametrize("work_path", [False, True])
def test_knob_wide_bits(pp_raw, wbits, work_path):
    """FTS_WIDE_BITS=20/22: the per-proof bases' fixed-base tables with 20- or
    22-bit windows (the default picks 22 when the free HBM holds them): the same
    H'_i, com and x0 bytes and verdicts on both com paths; table_bytes follows"""
    env = dict(FTS_WIDE_BITS=wbits, FTS_LANES=1)
    if work_path:
        env["FTS_COM_FIXED_MAX"] = 0
    pp = _ctx(pp_raw, 32, **env)
    try:
        # 16-bit tables of the 2n + 6 bases (32 MiB each) + the n + 2 wide ones
        wide = (32 + 2) * (13 * (1 << 19) if wbits == 20 else 12 * (1 << 21)) * 64
        assert pp.table_bytes == (2 * 32 + 6) * 32 * (1 << 20) + wide, pp.table_bytes
        _golden_check(pp, 32, work_path)
    finally:
        pp.close()


@pytest.mark.parametrize("env", [dict(FTS_WAVE_PRIO="000000000000"), dict(FTS_WAVE_PRIO="333333333333"),
                                 dict(FTS_WORK_BS=256), dict(FTS_MSM_MAXC=12)])
def test_knob_wave_prio_and_work_bs(pp_raw, env):
    """FTS_WAVE_PRIO (the s_setprio level of each kernel group, device/wave_prio.hpp),
    FTS_WORK_BS (block size of the work path's per-proof latency kernels) and
    FTS_MSM_MAXC (the widest MSM window a plan takes) change scheduling and the MSM
    plan only: a tampered rp32 pass on the work path gives the same exact verdicts,
    and the golden vectors stay byte-exact"""
    pp = _ctx(pp_raw, 32, FTS_LANES=1, FTS_COM_FIXED_MAX=0, **env)
    try:
        (b, want), = _tampered_batches(pp, 1, 768, 0x9410)
        got = b.verify(want_status=True)
        assert (got == want).all(), np.nonzero(got != want)
        b.close()
        _golden_check(pp, 32, True)
    finally:
        pp.close()
        # the next context re-uploads the default priority table, block size and window cap
