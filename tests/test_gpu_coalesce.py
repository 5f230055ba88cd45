"""GPU: action calls coalesced into shared device passes (fts_api.cpp act_stage /
rp_dispatch / run_rp_groups).

Concurrent fts_transfer_verify_batch, fts_issue_verify_batch,
fts_actions_verify_batch and fts_request_verify_batch calls and a staged
range-proof batch are queued behind fts_debug_hold and verified as ONE pass: the
range proofs of all five calls in one batch check, each call's sigma proofs in
its own slot beside them.  Every call must get exactly the (status, fail_index)
it gets alone -- the reference verifies every action on its own
(core/common/validator.go:215-224):
- transfer/transfer.go:192-196: a TypeAndSum failure wins over its (here forged)
  range proofs, which leave the batch check (k_sig_exclude at pass offsets);
- issue/verifier.go:40-56: SameType first, then RangeCorrectness;
- rp/rangecorrectness.go:141-160: the first failing range proof and its index;
- deserialisation failures and 1-in/1-out transfers (no range proofs) beside them.
Also the context options (fts_ctx_create_opts: table budget, window width) and
two range-proof contexts plus an identity handle on one GPU."""
import os
import random
import threading

import numpy as np
import pytest

from oracle import bn254 as bn, der, zkat

pytestmark = pytest.mark.gpu

BITS = 16


def _tamper_rp(raw, j, fn):
    sig, rc = der.unmarshal_values(raw)
    proofs = zkat.rc_deserialize(rc)
    fn(proofs[j])
    return der.values([sig, zkat.rc_serialize(proofs)])


def _break_sigma(raw, cls):
    sig, rc = der.unmarshal_values(raw)
    s = cls.deserialize(sig)
    s.Chal = (s.Chal + 1) % bn.R
    return der.values([s.serialize(), rc])


def _t1(r):
    r.data.T1 = bn.g1_add(r.data.T1, bn.GEN)


def _l(q):
    def f(r):
        r.ipa.L[q] = bn.g1_add(r.ipa.L[q], bn.GEN)
    return f


def _one_lane(pp_raw):
    import fts_gpu
    old = os.environ.get("FTS_IDLE_GATHER_US")
    os.environ["FTS_IDLE_GATHER_US"] = "0"
    try:
        return fts_gpu.PublicParams(pp_raw, bit_length=BITS, device=0, lanes=1)
    finally:
        if old is None:
            os.environ.pop("FTS_IDLE_GATHER_US", None)
        else:
            os.environ["FTS_IDLE_GATHER_US"] = old


def _workload(pp, seed):
    import fts_gpu
    F = fts_gpu
    rng = random.Random(seed)
    T = b"EUR"

    def bf():
        return rng.randrange(bn.R).to_bytes(32, "big")

    def transfers(n, n_in=2, n_out=2):
        wit = []
        for _ in range(n):
            iv = [rng.getrandbits(BITS - 2) for _ in range(n_in)]
            tot = sum(iv)
            ov = [rng.randrange(tot + 1)] if n_out == 2 else []
            ov.append(tot - sum(ov))
            wit.append((T, iv, [bf() for _ in iv], ov, [bf() for _ in ov]))
        proofs = pp.prove_transfers_gpu(wit, seed=rng.getrandbits(40))
        return [([pp.token_commit(t, v, x) for v, x in zip(iv, ib)], [pp.token_commit(t, v, x) for v, x in zip(ov, ob)],
                 p) for (t, iv, ib, ov, ob), p in zip(wit, proofs)], wit

    def issues(n, m=4):
        wit = [(T, [rng.getrandbits(BITS) for _ in range(m)], [bf() for _ in range(m)]) for _ in range(n)]
        proofs = pp.prove_issues_gpu(wit, seed=rng.getrandbits(40))
        return [([pp.token_commit(t, v, x) for v, x in zip(vs, bs)], p) for (t, vs, bs), p in zip(wit, proofs)], wit

    # call A: 2-in/2-out transfers with every transfer failure class
    tA, wA = transfers(96)
    wantA = [(0, -1)] * len(tA)
    ins, outs, p = tA[5]  # output 0 committed to another value AND its range proof forged: TypeAndSum wins
    t, iv, ib, ov, ob = wA[5]
    tA[5] = (ins, [pp.token_commit(t, ov[0] + 1, ob[0]), outs[1]], _tamper_rp(p, 0, _t1))
    wantA[5] = (F.FTS_E_TAS_INVALID, -1)
    ins, outs, p = tA[17]  # challenge broken + range proof 1 forged
    tA[17] = (ins, outs, _tamper_rp(_break_sigma(p, zkat.TypeAndSumProof), 1, _l(2)))
    wantA[17] = (F.FTS_E_TAS_INVALID, -1)
    ins, outs, p = tA[40]
    tA[40] = (ins, outs, _tamper_rp(p, 1, _t1))
    wantA[40] = (F.FTS_E_RP_INVALID, 1)
    ins, outs, p = tA[41]
    tA[41] = (ins, outs, _tamper_rp(p, 0, _l(3)))
    wantA[41] = (F.FTS_E_IPA_INVALID, 0)
    ins, outs, p = tA[77]  # truncated proof bytes
    tA[77] = (ins, outs, p[:len(p) // 2])
    wantA[77] = (F.FTS_E_MALFORMED, -1)
    # call B: issues of 4 tokens
    iB, wB = issues(48)
    wantB = [(0, -1)] * len(iB)
    toks, p = iB[3]
    iB[3] = (toks, _tamper_rp(_break_sigma(p, zkat.SameType), 2, _t1))
    wantB[3] = (F.FTS_E_ST_INVALID, -1)
    toks, p = iB[20]
    t, vs, bs = wB[20]
    toks = list(toks)
    toks[2] = pp.token_commit(t, vs[2] ^ 1, bs[2])
    iB[20] = (toks, p)
    wantB[20] = (F.FTS_E_RP_INVALID, 2)
    toks, p = iB[31]
    iB[31] = (toks, _tamper_rp(p, 3, _l(1)))
    wantB[31] = (F.FTS_E_IPA_INVALID, 3)
    # call C: mixed -- 1-in/1-out transfers (no range proofs), 2-in/2-out, issues
    tC1, _ = transfers(12, 1, 1)
    tC2, _ = transfers(20)
    iC, _ = issues(8, 2)
    tC = tC1 + tC2
    wantC_t = [(0, -1)] * len(tC)
    ins, outs, p = tC[3]  # a 1-in/1-out transfer whose TypeAndSum fails
    tC[3] = (ins, outs, _break_sigma(p, zkat.TypeAndSumProof))
    wantC_t[3] = (F.FTS_E_TAS_INVALID, -1)
    ins, outs, p = tC[15]
    tC[15] = (ins, outs, _tamper_rp(p, 0, _t1))
    wantC_t[15] = (F.FTS_E_RP_INVALID, 0)
    wantC_i = [(0, -1)] * len(iC)
    # call D: raw TokenRequests, one transfer action each
    R = F.request
    tD, _ = transfers(24)
    wantD = [(0, -1, -1)] * len(tD)
    ins, outs, p = tD[9]
    tD[9] = (ins, outs, _tamper_rp(p, 1, _t1))
    wantD[9] = (F.FTS_E_RP_INVALID, 0, 1)
    reqs = []
    for i, (ins, outs, p) in enumerate(tD):
        ta = R.transfer_action([("%064x" % (2 * i + k), k, b"owner-%d" % i, c) for k, c in enumerate(ins)],
                               [(b"recipient-%d" % i, c) for c in outs], p)
        reqs.append(R.token_request([(R.TRANSFER, ta)], [b"\x30" * 72, b"\x30" * 72]))
    # call E: a staged range-proof batch with one bad proof
    vals = [rng.getrandbits(BITS) for _ in range(200)]
    proofs, coms = pp.prove_range_batch_gpu(vals, [bf() for _ in vals], seed=rng.getrandbits(40))
    r = zkat.RangeProof.deserialize(proofs[123])
    r.data.T1 = bn.g1_add(r.data.T1, bn.GEN)
    proofs[123] = r.serialize()
    wantE = [0] * len(proofs)
    wantE[123] = F.FTS_E_RP_INVALID
    return dict(A=(tA, wantA), B=(iB, wantB), C=(tC, iC, wantC_t, wantC_i), D=(reqs, wantD), E=(proofs, coms, wantE))


def _calls(pp, w):
    """the five calls as callables -> comparable results"""
    tA, _ = w["A"]
    iB, _ = w["B"]
    tC, iC, _, _ = w["C"]
    reqs, _ = w["D"]
    proofs, coms, _ = w["E"]
    bA, bC, bD = pp.prepare_transfers(tA), pp.prepare_actions(tC, iC), pp.prepare_requests(reqs)
    sE = pp.stage_range_proofs(proofs, coms)

    def lst(*arrs):
        return [list(zip(*[a.tolist() for a in arrs]))]
    return {
        "A": lambda: lst(*bA.verify()),
        "B": lambda: lst(*pp.verify_issues(iB)),
        "C": lambda: (lambda r: lst(r[0], r[1]) + lst(r[2], r[3]))(bC.verify()),
        "D": lambda: lst(*bD.verify()),
        "E": lambda: [[int(x) for x in sE.verify()]],
    }, sE


def _want(w):
    return {"A": [w["A"][1]], "B": [w["B"][1]], "C": [w["C"][2], w["C"][3]], "D": [w["D"][1]], "E": [w["E"][2]]}


def test_action_calls_share_one_pass_exact_verdicts(pp_raw):
    """five calls of four entry points held until all are queued: ONE device pass
    (dispatcher counters), every call's verdicts equal to its verdicts alone and to
    the tampering, twice (fresh RLC weights each pass)"""
    pp = _one_lane(pp_raw)
    try:
        w = _workload(pp, 0xC0A1E5)
        calls, staged = _calls(pp, w)
        want = _want(w)
        alone = {}
        for name, fn in calls.items():
            s0 = pp.dispatch_stats()
            alone[name] = fn()
            s1 = pp.dispatch_stats()
            assert s1[0] - s0[0] == 1 and s1[1] - s0[1] == 1, (name, s0, s1)  # its own pass
            assert alone[name] == want[name], name
        for rep in range(2):
            got = {}
            s0 = pp.dispatch_stats()
            pp.hold(len(calls))
            th = [threading.Thread(target=lambda n=n, f=f: got.__setitem__(n, f())) for n, f in calls.items()]
            for x in th:
                x.start()
            for x in th:
                x.join()
            s1 = pp.dispatch_stats()
            assert s1[0] - s0[0] == 1 and s1[1] - s0[1] == len(calls), (s0, s1)  # one pass, five calls
            assert s1[2] >= len(calls) and s1[3] - s0[3] == 4, (s0, s1)          # four of them action calls
            assert staged.merged() == len(calls)
            for name in calls:
                assert got[name] == alone[name], (rep, name)
        staged.close()
    finally:
        pp.close()


def test_action_calls_coalesce_under_load(pp_raw):
    """no hold, four lanes: 12 threads x 3 rounds of transfer / issue / mixed calls as
    they come -- whatever passes the dispatcher forms, every verdict is the call's own"""
    import fts_gpu
    pp = fts_gpu.PublicParams(pp_raw, bit_length=BITS, device=0)
    try:
        w = _workload(pp, 0x5EED5)
        calls, staged = _calls(pp, w)
        want = _want(w)
        names = list(calls)
        errs = []

        def run(t):
            for r in range(3):
                n = names[(t + r) % len(names)]
                if calls[n]() != want[n]:
                    errs.append((t, r, n))
        th = [threading.Thread(target=run, args=(t,)) for t in range(12)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs
        staged.close()
    finally:
        pp.close()


def test_ctx_opts_window_width_and_budget(pp_raw):
    """fts_ctx_create_opts: an explicit window width, and a table budget below the
    22-bit tables' size, give 20-bit tables (fts_pp_info.wide_bits / table_bytes);
    a budget that holds them gives 22; the verdicts are the golden ones either way"""
    import json
    from conftest import GOLDEN
    import fts_gpu
    with open(os.path.join(GOLDEN, "rp_golden.json")) as f:
        gold = [c for c in json.load(f) if c["bits"] == 32]
    status_of = {None: 0, "invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
                 "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}
    base = (2 * 32 + 6) * 32 * (1 << 20)
    w20, w22 = (32 + 2) * 13 * (1 << 19) * 64, (32 + 2) * 12 * (1 << 21) * 64
    for kw, wb in ((dict(wide_bits=20), 20), (dict(table_budget=base + w22 - 1), 20),
                   (dict(table_budget=base + w22), 22), (dict(wide_bits=22, lanes=2), 22)):
        pp = fts_gpu.PublicParams(pp_raw, bit_length=32, device=0, **kw)
        try:
            assert pp.wide_bits == wb, (kw, pp.wide_bits)
            assert pp.table_bytes == base + (w22 if wb == 22 else w20), (kw, pp.table_bytes)
            assert pp.lanes == kw.get("lanes", 4)
            st = pp.verify_range_proofs([bytes.fromhex(c["proof"]) for c in gold],
                                        [bytes.fromhex(c["commitment"]) for c in gold])
            assert [int(s) for s in st] == [status_of[c["expect"]] for c in gold], kw
        finally:
            pp.close()


def test_two_contexts_and_identity_handle_one_gpu(pp_raw):
    """a second 64-bit context beside a first (default budget: the first
    takes 22-bit tables, the second falls back to 20-bit) plus an idemix identity
    handle on the same GPU -- no ENOMEM, and both contexts verify at their full pass
    size (workspace reserved for 81,920-proof passes)"""
    import fts_gpu
    from fts_gpu import idemix
    from conftest import GOLDEN
    a = fts_gpu.PublicParams(pp_raw, device=0)
    b = fts_gpu.PublicParams(pp_raw, device=0)
    ipk_path = os.path.join(GOLDEN, "idemix", "bn254_charlie", "IssuerPublicKey")
    h = None
    try:
        assert a.wide_bits in (20, 22) and b.wide_bits in (20, 22)
        a.reserve()
        b.reserve()
        with open(ipk_path, "rb") as f:
            h = idemix.IdentityVerifier(f.read(), device=0, curve=idemix.FTS_CURVE_BN254)
        rng = random.Random(0x2C7)
        vals = [rng.getrandbits(64) for _ in range(64)]
        bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(64)]
        proofs, coms = a.prove_range_batch_gpu(vals, bfs, seed=0x2C7)
        for pp in (a, b):
            assert not any(int(s) for s in pp.verify_range_proofs(proofs, coms))
    finally:
        if h is not None:
            h.close()
        b.close()
        a.close()
