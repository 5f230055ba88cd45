"""GPU parity at BASELINE config C5's full per-GPU size: 4,096 2-in/2-out
transfers + 1,024 issues with 16 outputs at 32-bit range (24,576 range proofs)
in ONE fts_actions_verify_batch call, ~1 % of the actions tampered.

The pass is above FTS_COM_FIXED_MAX, so it takes the work path (Horner + joint
GLV com chain); honest and tampered range proofs share one random linear
combination, whose failure runs the group test; range proofs of actions whose
sigma proof fails are excluded from it (k_sig_exclude).  Reference behaviour at
stake (token/core/zkatdlog/nogh/v1/crypto/...):
- transfer/transfer.go:192-196: a TypeAndSum failure wins, its range proofs are
  never reached (here they are forged too);
- issue/verifier.go:40-56: SameType first, then RangeCorrectness;
- rp/rangecorrectness.go:141-160: the first failing range proof and its index.
Every (status, fail index) is asserted at its position against the tampering,
every tampered action and a sample of honest ones against the reference-order C
restatement (oracle/c/ref_verify.c), and one action per tamper class against the
Python oracle (oracle/zkat.py)."""
import random

import numpy as np
import pytest

from oracle import bn254 as bn, cref, der, zkat

pytestmark = pytest.mark.gpu

N_TR, N_IS, BITS = 4096, 1024, 32


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


def _t2(r):
    r.data.T2 = bn.g1_add(r.data.T2, bn.GEN)


def _l(q):
    def f(r):
        r.ipa.L[q] = bn.g1_add(r.ipa.L[q], bn.GEN)
    return f


@pytest.fixture(scope="module")
def c5(gpu_pp):
    import fts_gpu
    pp = gpu_pp(BITS)
    rng = random.Random(0xC5C5)
    T = b"USD"

    def bf():
        return rng.randrange(bn.R).to_bytes(32, "big")

    twit = []
    for _ in range(N_TR):
        a, b = rng.getrandbits(BITS - 1), rng.getrandbits(BITS - 1)
        c = rng.randrange(a + b + 1)
        twit.append((T, [a, b], [bf(), bf()], [c, a + b - c], [bf(), bf()]))
    iwit = [(T, [rng.getrandbits(BITS) for _ in range(16)], [bf() for _ in range(16)]) for _ in range(N_IS)]
    tproofs = pp.prove_transfers_gpu(twit, seed=0xC51)
    iproofs = pp.prove_issues_gpu(iwit, seed=0xC52)
    transfers = [([pp.token_commit(t, v, x) for v, x in zip(iv, ib)], [pp.token_commit(t, v, x) for v, x in zip(ov, ob)],
                  p) for (t, iv, ib, ov, ob), p in zip(twit, tproofs)]
    issues = [([pp.token_commit(t, v, x) for v, x in zip(vs, bs)], p) for (t, vs, bs), p in zip(iwit, iproofs)]
    want_t = [(0, -1)] * N_TR
    want_i = [(0, -1)] * N_IS
    cls_t, cls_i = {}, {}
    bad_t = sorted(rng.sample(range(N_TR), N_TR // 100))
    bad_i = sorted(rng.sample(range(N_IS), N_IS // 100))
    for q, i in enumerate(bad_t):
        ins, outs, p = transfers[i]
        t, iv, ib, ov, ob = twit[i]
        kind, j = q % 5, rng.randrange(2)
        if kind == 0:    # output 0 committed to another value, its range proof forged too: TypeAndSum wins
            outs = [pp.token_commit(t, ov[0] + 1, ob[0]), outs[1]]
            p = _tamper_rp(p, 0, _t1)
            w = (fts_gpu.FTS_E_TAS_INVALID, -1)
        elif kind == 1:  # TypeAndSum challenge broken AND range proof j's L_2 forged
            p = _tamper_rp(_break_sigma(p, zkat.TypeAndSumProof), j, _l(2))
            w = (fts_gpu.FTS_E_TAS_INVALID, -1)
        elif kind == 2:  # T1 of range proof j
            p = _tamper_rp(p, j, _t1)
            w = (fts_gpu.FTS_E_RP_INVALID, j)
        elif kind == 3:  # L_3 of range proof j
            p = _tamper_rp(p, j, _l(3))
            w = (fts_gpu.FTS_E_IPA_INVALID, j)
        else:            # both range proofs forged: the first one fails
            p = _tamper_rp(_tamper_rp(p, 1, _t2), 0, _l(0))
            w = (fts_gpu.FTS_E_IPA_INVALID, 0)
        transfers[i] = (ins, outs, p)
        want_t[i] = w
        cls_t.setdefault(kind, i)
    for q, i in enumerate(bad_i):
        toks, p = issues[i]
        t, vs, bs = iwit[i]
        kind, j = q % 4, rng.randrange(3)
        if kind == 0:    # SameType challenge broken AND range proof 3 forged: SameType wins
            p = _tamper_rp(_break_sigma(p, zkat.SameType), 3, _t1)
            w = (fts_gpu.FTS_E_ST_INVALID, -1)
        elif kind == 1:  # token j committed to another value
            toks = list(toks)
            toks[j] = pp.token_commit(t, vs[j] ^ 1, bs[j])
            w = (fts_gpu.FTS_E_RP_INVALID, j)
        elif kind == 2:  # L_1 of range proof j
            p = _tamper_rp(p, j, _l(1))
            w = (fts_gpu.FTS_E_IPA_INVALID, j)
        else:            # T2 of range proof j
            p = _tamper_rp(p, j, _t2)
            w = (fts_gpu.FTS_E_RP_INVALID, j)
        issues[i] = (toks, p)
        want_i[i] = w
        cls_i.setdefault(kind, i)
    return dict(pp=pp, transfers=transfers, issues=issues, want_t=want_t, want_i=want_i, bad_t=bad_t, bad_i=bad_i,
                cls_t=cls_t, cls_i=cls_i)


def test_c5_full_size_one_call_exact_verdicts(c5):
    pp = c5["pp"]
    st_t, fi_t, st_i, fi_i = pp.verify_actions(c5["transfers"], c5["issues"])
    tim = pp.last_timings_ex()
    got_t = list(zip(st_t.tolist(), fi_t.tolist()))
    got_i = list(zip(st_i.tolist(), fi_i.tolist()))
    assert got_t == c5["want_t"], [i for i, (a, b) in enumerate(zip(got_t, c5["want_t"])) if a != b][:10]
    assert got_i == c5["want_i"], [i for i, (a, b) in enumerate(zip(got_i, c5["want_i"])) if a != b][:10]
    # the pass took the work path and the batch check's group test
    assert "k_rp_com_var" in tim and "k_rp_fixed_exact" in tim, sorted(tim)
    assert any(k.startswith("fb:") for k in tim), sorted(tim)
    # the same verdicts again (idempotence; fresh RLC weights)
    s2 = pp.verify_actions(c5["transfers"], c5["issues"])
    assert (s2[0] == st_t).all() and (s2[1] == fi_t).all() and (s2[2] == st_i).all() and (s2[3] == fi_i).all()


def test_c5_reference_order_oracle(c5, oracle_pp):
    """every tampered action and 32 honest ones through the reference-order C
    restatement; one action per tamper class through the Python oracle"""
    opp = oracle_pp.with_bit_length(BITS)
    rng = random.Random(5)
    ti = c5["bad_t"] + rng.sample([i for i in range(N_TR) if i not in set(c5["bad_t"])], 24)
    ii = c5["bad_i"] + rng.sample([i for i in range(N_IS) if i not in set(c5["bad_i"])], 8)
    acts = [("transfer",) + tuple(c5["transfers"][i]) for i in ti] + \
        [("issue", []) + tuple(c5["issues"][i]) for i in ii]
    got = cref.action_verify_many(opp, acts, threads=8)
    want = [c5["want_t"][i] for i in ti] + [c5["want_i"][i] for i in ii]
    assert got == want
    import fts_gpu
    for i in c5["cls_t"].values():
        ins, outs, p = c5["transfers"][i]
        err, idx = zkat.transfer_verify(opp, [bn.g1_from_bytes(x) for x in ins], [bn.g1_from_bytes(x) for x in outs], p)
        s, f = c5["want_t"][i]
        assert fts_gpu.transfer_message(s, f) == err and f == idx, i
    for i in c5["cls_i"].values():
        toks, p = c5["issues"][i]
        err, idx = zkat.issue_verify(opp, [bn.g1_from_bytes(x) for x in toks], p)
        s, f = c5["want_i"][i]
        assert fts_gpu.issue_message(s, f) == err and f == idx, i
