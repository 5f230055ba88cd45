"""GPU parity: transfer (TypeAndSum + RangeCorrectness, transfer/transfer.go:49-197)
and issue (SameType + RangeCorrectness, issue/verifier.go:24-57) batch
verification against the oracle, including the reference's error precedence."""
import json
import os

import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, der, zkat

pytestmark = pytest.mark.gpu


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


TRANSFERS = _load("transfer_golden.json")
ISSUES = _load("issue_golden.json")


@pytest.mark.parametrize("bits", [8, 16])
def test_golden_transfers(gpu_pp, bits):
    import fts_gpu
    cases = [c for c in TRANSFERS if c["bits"] == bits]
    pp = gpu_pp(bits)
    items = [([bytes.fromhex(h) for h in c["inputs"]], [bytes.fromhex(h) for h in c["outputs"]],
              bytes.fromhex(c["proof"])) for c in cases]
    st, fi = pp.verify_transfers(items)
    for c, s, i in zip(cases, st, fi):
        assert fts_gpu.transfer_message(int(s), int(i)) == c["expect"], c["name"]


@pytest.mark.parametrize("bits", [8, 16])
def test_golden_issues(gpu_pp, bits):
    import fts_gpu
    cases = [c for c in ISSUES if c["bits"] == bits]
    pp = gpu_pp(bits)
    st, fi = pp.verify_issues([([bytes.fromhex(h) for h in c["tokens"]], bytes.fromhex(c["proof"])) for c in cases])
    for c, s, i in zip(cases, st, fi):
        assert fts_gpu.issue_message(int(s), int(i)) == c["expect"], c["name"]


def _bf(i):
    return (0x5EED + 17 * i).to_bytes(32, "big")


RP_STATUS = {"invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
             "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}


def oracle_status(err, idx, prefix=""):
    """reference error chain -> (fts_status, fail index)"""
    if err is None:
        return (0, -1)
    e = err[len(prefix):] if prefix and err.startswith(prefix) else err
    if e.endswith("invalid sum and type proof"):
        return (8, -1)
    if e.endswith("invalid same type proof"):
        return (9, -1)
    if e == "invalid range proof":
        return (7, -1)
    if e.startswith("invalid range proof at index"):
        inner = e.split(": ", 1)[1]
        return (RP_STATUS[inner], idx)
    return (1, -1)  # deserialisation / panic


def test_transfer_batch_mixed(gpu_pp, oracle_pp):
    """A batch of product-prover transfers with every failure class, each
    verdict equal to the oracle's (reference) verdict."""
    import fts_gpu
    bits = 16
    pp = gpu_pp(bits)
    opp = oracle_pp.with_bit_length(bits)
    T = b"ABC"
    items, expect = [], []

    def add(inv, outv, proof_outv=None, mutate=None, seed=1):
        ib = [_bf(seed * 10 + j) for j in range(len(inv))]
        ob = [_bf(seed * 10 + 5 + j) for j in range(len(outv))]
        ins = [pp.token_commit(T, v, b) for v, b in zip(inv, ib)]
        outs = [pp.token_commit(T, v, b) for v, b in zip(outv, ob)]
        proof = pp.prove_transfer(T, inv, ib, proof_outv or outv, ob, seed)
        if mutate:
            proof = mutate(proof)
        items.append((ins, outs, proof))
        try:
            err, idx = zkat.transfer_verify(opp, [bn.g1_from_bytes(x) for x in ins], [bn.g1_from_bytes(x) for x in outs],
                                            proof)
        except zkat.Malformed:
            err, idx = "malformed", -1
        expect.append(oracle_status(err, idx))

    add([100, 200], [250, 50], seed=1)                          # honest
    add([1, 2, 3], [6], seed=2)                                 # honest 3-in/1-out
    add([5], [5], seed=3)                                       # 1-in/1-out: no range proofs
    add([100, 200], [250, 51], seed=4)                          # wrong sum
    add([70000 - 65536, 1], [70000 - 65536 - 10, 11], proof_outv=None, seed=5)

    def drop_rc(p):
        t, rc = der.unmarshal_values(p)
        return der.values([t, b""])
    add([10, 20], [15, 15], mutate=drop_rc, seed=6)             # no range proofs -> "invalid range proof"

    def swap_rp(p):
        t, rc = der.unmarshal_values(p)
        rps = der.unmarshal_values(der.unmarshal_values(rc)[0])
        return der.values([t, der.values([der.values([rps[1], rps[0]])])])
    add([10, 20], [12, 18], mutate=swap_rp, seed=7)             # range proof at index 0 invalid

    def break_chal(p):
        t, rc = der.unmarshal_values(p)
        s = zkat.TypeAndSumProof.deserialize(t)
        s.Chal = (s.Chal + 1) % bn.R
        return der.values([s.serialize(), rc])
    add([10, 20], [12, 18], mutate=break_chal, seed=8)

    def nil_tas(p):
        t, rc = der.unmarshal_values(p)
        return der.values([b"", rc])
    add([5], [5], mutate=nil_tas, seed=9)                       # all-nil TypeAndSum: invalid sum and type

    add([10, 20], [30, 0], mutate=lambda p: p[:-7], seed=10)    # truncated
    st, fi = pp.verify_transfers(items)
    assert [(int(s), int(i)) for s, i in zip(st, fi)] == expect


def test_issue_batch_mixed(gpu_pp, oracle_pp):
    import fts_gpu
    bits = 8
    pp = gpu_pp(bits)
    opp = oracle_pp.with_bit_length(bits)
    T = b"USD"
    items, expect = [], []
    for seed, vals, mut in ((1, [1, 2, 3], None), (2, [255], None), (3, [256, 1], None), (4, [9, 9], "swap")):
        bfs = [_bf(seed * 10 + j) for j in range(len(vals))]
        toks = [pp.token_commit(T, v, b) for v, b in zip(vals, bfs)]
        proof = pp.prove_issue(T, vals, bfs, seed)
        if mut == "swap":
            toks = toks[::-1]
            toks[0] = pp.token_commit(T, 10, bfs[1])
        items.append((toks, proof))
        err, idx = zkat.issue_verify(opp, [bn.g1_from_bytes(x) for x in toks], proof)
        expect.append(oracle_status(err, idx, "invalid issue proof: "))
    st, fi = pp.verify_issues(items)
    assert [(int(s), int(i)) for s, i in zip(st, fi)] == expect


def test_reference_shaped_transfer_api(gpu_pp):
    import fts_gpu
    pp = gpu_pp(16)
    ib, ob = [_bf(1), _bf(2)], [_bf(3), _bf(4)]
    ins = [pp.token_commit(b"ABC", v, b) for v, b in zip([220, 60], ib)]
    outs = [pp.token_commit(b"ABC", v, b) for v, b in zip([260, 20], ob)]
    fts_gpu.TransferVerifier(ins, outs, pp).Verify(pp.prove_transfer(b"ABC", [220, 60], ib, [260, 20], ob, 1))
    with pytest.raises(fts_gpu.VerifyError) as e:
        fts_gpu.TransferVerifier(ins, outs, pp).Verify(pp.prove_transfer(b"ABC", [220, 60], ib, [261, 20], ob, 1))
    assert "invalid transfer proof: invalid sum and type proof" in str(e.value)


def test_mixed_actions_one_pass(gpu_pp, oracle_pp):
    """BASELINE config C5 shape: issues with 16 outputs at 32-bit range plus
    2-in/2-out transfers, verified in ONE device pass
    (fts_actions_verify_batch).  Every verdict equals the oracle's
    (reference) verdict and the separate transfer / issue calls."""
    bits = 32
    pp = gpu_pp(bits)
    opp = oracle_pp.with_bit_length(bits)
    T = b"USD"
    transfers, t_expect = [], []
    for seed in range(1, 5):
        inv = [1000 * seed + 7, 50 * seed]
        outv = [inv[0] - seed, inv[1] + seed] if seed != 3 else [inv[0], inv[1] + 1]  # seed 3: wrong sum
        ib = [_bf(seed * 10 + j) for j in range(2)]
        ob = [_bf(seed * 10 + 5 + j) for j in range(2)]
        ins = [pp.token_commit(T, v, b) for v, b in zip(inv, ib)]
        outs = [pp.token_commit(T, v, b) for v, b in zip(outv, ob)]
        proof = pp.prove_transfer(T, inv, ib, outv, ob, seed)
        transfers.append((ins, outs, proof))
        err, idx = zkat.transfer_verify(opp, [bn.g1_from_bytes(x) for x in ins], [bn.g1_from_bytes(x) for x in outs],
                                        proof)
        t_expect.append(oracle_status(err, idx))
    issues, i_expect = [], []
    for seed in (21, 22):
        vals = [(seed * 7919 + 104729 * j) % (1 << 32) for j in range(16)]
        bfs = [_bf(seed * 100 + j) for j in range(16)]
        toks = [pp.token_commit(T, v, b) for v, b in zip(vals, bfs)]
        proof = pp.prove_issue(T, vals, bfs, seed)
        if seed == 22:  # token 5 committed to another value -> its range proof fails
            toks[5] = pp.token_commit(T, vals[5] + 1, bfs[5])
        issues.append((toks, proof))
        err, idx = zkat.issue_verify(opp, [bn.g1_from_bytes(x) for x in toks], proof)
        i_expect.append(oracle_status(err, idx, "invalid issue proof: "))
    st_t, fi_t, st_i, fi_i = pp.verify_actions(transfers, issues)
    assert [(int(s), int(i)) for s, i in zip(st_t, fi_t)] == t_expect
    assert [(int(s), int(i)) for s, i in zip(st_i, fi_i)] == i_expect
    assert t_expect[2][0] == 8 and t_expect[0] == (0, -1) and i_expect[0] == (0, -1) and i_expect[1][0] != 0
    s2, f2 = pp.verify_transfers(transfers)
    s3, f3 = pp.verify_issues(issues)
    assert (s2 == st_t).all() and (f2 == fi_t).all() and (s3 == st_i).all() and (f3 == fi_i).all()
