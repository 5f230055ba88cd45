"""GPU parity at the headline shapes (BASELINE configs C1/C4 and C5).

- headline_golden.json (oracle-made, tests/golden/make_golden_headline.py):
  64-bit 2-in/2-out transfers (honest, wrong sum, range failure at index 1,
  tampered T1 / L_3 / Delta / Right, and the reference's TypeAndSum negative
  cases of typeandsum_test.go:87-142: wrong type, wrong values, wrong blinding
  factors) and issues with 16 outputs at 32 bits (honest, a token committed to
  another value, tampered SameType challenge, tampered L_2 of proof 11).
- C4 per-GPU batch: 8,192 64-bit 2-in/2-out transfers (16,384 rp64 + 8,192
  TypeAndSum, BASELINE configs[3] / 8 GPUs) with ~1 % tampered: every verdict and
  fail index equals the one the tampering implies, and a sample equals the
  oracle's (reference) verdict.
All through the C-ABI (fts_transfer_verify_batch / fts_issue_verify_batch)."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, der, zkat

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "headline_golden.json")) as _f:
    HEAD = json.load(_f)


def test_headline_transfers_64bit(gpu_pp):
    import fts_gpu
    pp = gpu_pp(64)
    cases = HEAD["transfers"]
    items = [([bytes.fromhex(h) for h in c["inputs"]], [bytes.fromhex(h) for h in c["outputs"]],
              bytes.fromhex(c["proof"])) for c in cases]
    st, fi = pp.verify_transfers(items)
    got = [fts_gpu.transfer_message(int(s), int(i)) for s, i in zip(st, fi)]
    assert got == [c["expect"] for c in cases]
    assert [int(i) for i in fi] == [c["index"] for c in cases]
    # the same items one at a time (a batch of one must not change any verdict)
    for c, it in zip(cases[:4], items[:4]):
        s1, f1 = pp.verify_transfers([it])
        assert fts_gpu.transfer_message(int(s1[0]), int(f1[0])) == c["expect"], c["name"]


def test_headline_issues_16x32bit(gpu_pp):
    import fts_gpu
    pp = gpu_pp(32)
    cases = HEAD["issues"]
    st, fi = pp.verify_issues([([bytes.fromhex(h) for h in c["tokens"]], bytes.fromhex(c["proof"])) for c in cases])
    assert [fts_gpu.issue_message(int(s), int(i)) for s, i in zip(st, fi)] == [c["expect"] for c in cases]
    # the mixed entry point (one device pass for issues + transfers) gives the same verdicts
    s2, f2, s3, f3 = pp.verify_actions([], [([bytes.fromhex(h) for h in c["tokens"]], bytes.fromhex(c["proof"]))
                                            for c in cases])
    assert (s3 == st).all() and (f3 == fi).all()


def _tamper_rp(raw, j, fn):
    sig, rc = der.unmarshal_values(raw)
    proofs = zkat.rc_deserialize(rc)
    fn(proofs[j])
    return der.values([sig, zkat.rc_serialize(proofs)])


def test_c4_batch_8192_transfers_1pct_tampered(gpu_pp, oracle_pp):
    """BASELINE configs[3] per GPU: 8,192 2-in/2-out 64-bit transfers in ONE
    fts_transfer_verify_batch call, ~1 % tampered in four ways.  Exact positions,
    classes and fail indices; a sample re-verified by the oracle."""
    import fts_gpu
    pp = gpu_pp(64)
    rng = random.Random(0xF7A50004)
    n = 8192
    T = b"ABC"
    wit = []
    for _ in range(n):
        a, b = rng.getrandbits(62), rng.getrandbits(62)
        c = rng.randrange(a + b + 1)
        wit.append((T, [a, b], [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(2)], [c, a + b - c],
                    [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(2)]))
    proofs = pp.prove_transfers_gpu(wit, seed=0xC4)
    items = []
    for (t, iv, ib, ov, ob), p in zip(wit, proofs):
        items.append(([pp.token_commit(t, v, x) for v, x in zip(iv, ib)],
                      [pp.token_commit(t, v, x) for v, x in zip(ov, ob)], p))
    want_st = np.zeros(n, dtype=np.int32)
    want_fi = np.full(n, -1, dtype=np.int32)
    bad = sorted(rng.sample(range(n), n // 100))
    G = bn.GEN
    for q, i in enumerate(bad):
        ins, outs, p = items[i]
        kind, j = q % 4, rng.randrange(2)
        if kind == 0:    # T1 of range proof j -> "invalid range proof at index j: invalid range proof"
            p = _tamper_rp(p, j, lambda r: setattr(r.data, "T1", bn.g1_add(r.data.T1, G)))
            want_st[i], want_fi[i] = fts_gpu.FTS_E_RP_INVALID, j
        elif kind == 1:  # L_j of range proof j -> "... invalid IPA"
            p = _tamper_rp(p, j, lambda r: r.ipa.L.__setitem__(2, bn.g1_add(r.ipa.L[2], G)))
            want_st[i], want_fi[i] = fts_gpu.FTS_E_IPA_INVALID, j
        elif kind == 2:  # TypeAndSum challenge -> "invalid sum and type proof"
            tas, rc = der.unmarshal_values(p)
            s = zkat.TypeAndSumProof.deserialize(tas)
            s.Chal = (s.Chal + 1) % bn.R
            p = der.values([s.serialize(), rc])
            want_st[i] = fts_gpu.FTS_E_TAS_INVALID
        else:            # outputs swapped: the TypeAndSum transcript changes
            outs = outs[::-1]
            want_st[i] = fts_gpu.FTS_E_TAS_INVALID
        items[i] = (ins, outs, p)
    st, fi = pp.verify_transfers(items)
    assert (st == want_st).all(), np.nonzero(st != want_st)[0][:10]
    assert (fi == want_fi).all(), np.nonzero(fi != want_fi)[0][:10]
    # reference verdicts (oracle) on a sample: two honest + one of each tampering class
    sample = [0, n - 1] + bad[:4]
    for i in sample:
        ins, outs, p = items[i]
        err, idx = zkat.transfer_verify(oracle_pp, [bn.g1_from_bytes(x) for x in ins],
                                        [bn.g1_from_bytes(x) for x in outs], p)
        assert fts_gpu.transfer_message(int(st[i]), int(fi[i])) == err and int(fi[i]) == idx, i
