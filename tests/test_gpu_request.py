"""GPU: raw TokenRequest ingest (fts_request_verify_batch) -- the
deserialisation + ZK half of Validator.VerifyTokenRequestFromRaw
(core/common/validator.go:78-130) over one device pass per batch.

Requests are assembled (fts_gpu.request, the reference's proto layout) from the
golden transfer / issue proofs whose verdicts the oracle pins
(tests/golden/make_golden.py); the expected request verdict is the first
failing action in the reference's order -- every issue, then every transfer
(validator.go:116-126) -- with deserialisation failures first."""
import json
import os
import random

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return {c["name"]: c for c in json.load(f)}


T = _load("transfer_golden.json")
I = _load("issue_golden.json")


def _status(F, msg, issue):
    """golden reference message -> (fts_status, fail index) via the verdict maps the
    action tests already pin"""
    if msg is None:
        return F.FTS_OK, -1
    table = {
        "invalid transfer proof: invalid sum and type proof": (F.FTS_E_TAS_INVALID, -1),
        "invalid issue proof: invalid same type proof": (F.FTS_E_ST_INVALID, -1),
        "invalid range proof at index 0: invalid range proof": (F.FTS_E_RP_INVALID, 0),
        "invalid issue proof: invalid range proof at index 0: invalid range proof": (F.FTS_E_RP_INVALID, 0),
    }
    return table[msg]


def _transfer(F, name, owner=b"bob"):
    c = T[name]
    ins = [("tx-%s-%d" % (name, k), k, b"alice", bytes.fromhex(h)) for k, h in enumerate(c["inputs"])]
    outs = [(owner, bytes.fromhex(h)) for h in c["outputs"]]
    return (F.request.TRANSFER, F.request.transfer_action(ins, outs, bytes.fromhex(c["proof"]))), \
        _status(F, c["expect"], False)


def _issue(F, name):
    c = I[name]
    outs = [(b"bob", bytes.fromhex(h)) for h in c["tokens"]]
    return (F.request.ISSUE, F.request.issue_action(b"issuer", outs, bytes.fromhex(c["proof"]))), \
        _status(F, c["expect"], True)


def _expect(F, actions):
    """(status, fail_action, fail_index) of a request of (action, verdict) pairs"""
    order = [i for i, ((t, _), _) in enumerate(actions) if t == F.request.ISSUE] + \
            [i for i, ((t, _), _) in enumerate(actions) if t == F.request.TRANSFER]
    for i in order:
        st, fx = actions[i][1]
        if st != F.FTS_OK:
            return st, i, fx
    return F.FTS_OK, -1, -1


def _req(F, actions):
    return F.request.token_request([a for a, _ in actions], [b"sig"])


def test_requests_golden_mix(gpu_pp):
    import fts_gpu as F
    pp = gpu_pp(16)
    tr_names = ["honest_2in_2out", "wrong_sum", "ownership_1in_1out", "honest_3in_1out"]
    is_names = ["honest_2", "tampered_challenge"]
    cases = [
        [_issue(F, "honest_2"), _transfer(F, "honest_2in_2out")],
        [_transfer(F, "wrong_sum"), _issue(F, "tampered_challenge")],      # issue verdict wins
        [_transfer(F, "honest_3in_1out"), _transfer(F, "wrong_sum")],
        [_transfer(F, "ownership_1in_1out", owner=b"")],                     # redeem-shaped output
        [_issue(F, "honest_2"), _issue(F, "tampered_challenge"), _transfer(F, "wrong_sum")],
        [],
    ]
    rng = random.Random(0x7E0)
    for _ in range(150):  # enough requests for the multi-threaded host decode
        acts = [_transfer(F, rng.choice(tr_names)) if rng.random() < 0.7 else _issue(F, rng.choice(is_names))
                for _ in range(rng.randint(1, 4))]
        cases.append(acts)
    raws = [_req(F, a) for a in cases]
    st, fa, fi = pp.verify_requests(raws)
    for k, acts in enumerate(cases):
        assert (int(st[k]), int(fa[k]), int(fi[k])) == _expect(F, acts), k
    assert int(st[0]) == F.FTS_OK and int(st[1]) == F.FTS_E_ST_INVALID and int(fa[1]) == 1


def test_requests_structural_and_malformed(gpu_pp):
    import fts_gpu as F
    R = F.request
    pp = gpu_pp(16)
    honest, _ = _transfer(F, "honest_2in_2out")
    wrong, _ = _transfer(F, "wrong_sum")
    tampered, _ = _issue(F, "tampered_challenge")
    c = T["honest_2in_2out"]
    no_inputs = (R.TRANSFER, R.transfer_action([], [(b"b", bytes.fromhex(h)) for h in c["outputs"]],
                                               bytes.fromhex(c["proof"])))
    off_curve = R.g1(b"\x01" + b"\x00" * 63)
    bad_out = R.field_bytes(2, R.msg(1, R.opt_bytes(1, b"b") + R.msg(2, off_curve)))
    bad_g1 = (R.TRANSFER, honest[1] + bad_out)
    reqs = [
        # structurally invalid transfer after an honest one
        ([honest, no_inputs, wrong], (F.FTS_E_ACTION_INVALID, 1, -1)),
        # a failing proof before the invalid action is reported first
        ([wrong, no_inputs], (F.FTS_E_TAS_INVALID, 0, -1)),
        # issues go first even when listed last
        ([no_inputs, tampered], (F.FTS_E_ST_INVALID, 1, -1)),
        # deserialisation precedes every proof (DeserializeActions)
        ([tampered, bad_g1], (F.FTS_E_MALFORMED, 1, -1)),
        ([honest, (7, honest[1])], (F.FTS_E_MALFORMED, 1, -1)),
        # a proof that does not parse is the action's own verdict
        ([honest, (R.TRANSFER, R.transfer_action(
            [("t", 0, b"a", bytes.fromhex(h)) for h in c["inputs"]],
            [(b"b", bytes.fromhex(h)) for h in c["outputs"]], b"\x30\x03\x02\x01"))], (F.FTS_E_MALFORMED, 1, -1)),
        ([honest], (F.FTS_OK, -1, -1)),
    ]
    raws = [R.token_request(a, [b"s"]) for a, _ in reqs] + [b"", b"\xff\xff"]
    st, fa, fi = pp.verify_requests(raws)
    got = [(int(s), int(a), int(i)) for s, a, i in zip(st, fa, fi)]
    assert got[:len(reqs)] == [e for _, e in reqs]
    assert got[len(reqs):] == [(F.FTS_E_MALFORMED, -1, -1)] * 2


def test_requests_range_failure_index(gpu_pp):
    import fts_gpu as F
    pp = gpu_pp(8)
    acts = [_transfer(F, "out_of_range_8bit")]
    iss = [_issue(F, "out_of_range_8bit")]
    st, fa, fi = pp.verify_requests([_req(F, acts), _req(F, acts + iss), _req(F, [])])
    assert (int(st[0]), int(fa[0]), int(fi[0])) == (F.FTS_E_RP_INVALID, 0, 0)
    assert (int(st[1]), int(fa[1]), int(fi[1])) == (F.FTS_E_RP_INVALID, 1, 0)   # the issue (index 1) first
    assert (int(st[2]), int(fa[2])) == (F.FTS_OK, -1)


def test_requests_match_action_batch(gpu_pp):
    """the ingest path and the typed action batch give the same action verdicts"""
    import fts_gpu as F
    pp = gpu_pp(16)
    names = ["honest_2in_2out", "wrong_sum", "ownership_1in_1out", "honest_3in_1out"]
    raws, items = [], []
    for nm in names * 20:
        a, _ = _transfer(F, nm)
        raws.append(F.request.token_request([a], [b"s"]))
        cc = T[nm]
        items.append(([bytes.fromhex(h) for h in cc["inputs"]], [bytes.fromhex(h) for h in cc["outputs"]],
                      bytes.fromhex(cc["proof"])))
    st, fa, fi = pp.verify_requests(raws)
    st2, fi2 = pp.verify_transfers(items)
    assert list(st) == list(st2) and list(fi) == list(fi2)
    assert all(int(a) == (0 if s else -1) for s, a in zip(st, fa))
