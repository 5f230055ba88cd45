"""CPU: the C-ABI library loads, exports every symbol include/fts_gpu.h
declares, parses the public parameters, and its host prover produces
reference-format proofs that the independent oracle accepts (and rejects when
the statement is false) — no GPU compute here."""
import os
import re

import pytest

from conftest import ROOT

from oracle import bn254 as bn, zkat


def _header_functions():
    with open(os.path.join(ROOT, "include", "fts_gpu.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(fts_\w+)\s*\(", src, re.M)))


def test_exports_every_header_symbol():
    from fts_gpu import _lib as L
    names = _header_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(L.lib, n), n
    assert set(names) == set(L.EXPORTED)


def test_status_strings():
    from fts_gpu import _lib as L
    assert L.status_str(L.FTS_E_RP_INVALID) == "invalid range proof"
    assert L.status_str(L.FTS_E_IPA_INVALID) == "invalid IPA"
    assert L.status_str(L.FTS_E_IPA_NIL) == "invalid IPA proof: nil elements"
    assert L.status_str(L.FTS_E_IPA_LEN) == "invalid IPA proof"
    assert L.status_str(L.FTS_E_RP_NIL) == "invalid range proof: nil elements"
    assert L.status_str(L.FTS_E_TAS_INVALID) == "invalid sum and type proof"
    assert L.status_str(L.FTS_E_ST_INVALID) == "invalid same type proof"


def test_messages_match_reference_tests():
    """transfer_test.go:69,82 and the issue chain (issue/verifier.go:40-56)."""
    import fts_gpu as F
    assert F.transfer_message(F.FTS_E_TAS_INVALID, -1) == "invalid transfer proof: invalid sum and type proof"
    assert F.transfer_message(F.FTS_E_RP_INVALID, 0) == "invalid range proof at index 0: invalid range proof"
    assert F.issue_message(F.FTS_E_ST_INVALID, -1) == "invalid issue proof: invalid same type proof"
    assert F.transfer_message(F.FTS_OK, -1) is None


def test_host_context_info(host_pp):
    pp = host_pp(64)
    assert (pp.bit_length, pp.rounds, pp.max_token) == (64, 6, (1 << 64) - 1)
    pp8 = host_pp(8)
    assert (pp8.bit_length, pp8.rounds) == (8, 3)


def test_bad_public_params_rejected(pp_raw):
    import fts_gpu
    from fts_gpu import _lib as L
    with pytest.raises(L.FtsError):
        fts_gpu.PublicParams(pp_raw.replace(b"zkatdlog", b"fabtoken", 1), device=fts_gpu.FTS_DEVICE_NONE)
    with pytest.raises(L.FtsError):
        fts_gpu.PublicParams(b"{}", device=fts_gpu.FTS_DEVICE_NONE)
    with pytest.raises(L.FtsError):
        fts_gpu.PublicParams(pp_raw, bit_length=128, device=fts_gpu.FTS_DEVICE_NONE)


def test_verify_needs_device(host_pp):
    from fts_gpu import _lib as L
    with pytest.raises(L.FtsError):
        host_pp(8).verify_range_proofs([b"\x30\x00"], [bytes(64)])


@pytest.mark.parametrize("bits,value", [(8, 115), (8, 0), (16, 65535), (64, (1 << 64) - 1)])
def test_host_prover_accepted_by_oracle(host_pp, oracle_pp, bits, value):
    pp = host_pp(bits)
    opp = oracle_pp.with_bit_length(bits)
    bf = (0xABCDEF + value).to_bytes(32, "big")
    der_bytes, com = pp.prove_range(value, bf, seed=value + 1)
    V = bn.g1_from_bytes(com)
    assert V == bn.g1_add(bn.g1_mul(opp.ped[1], value), bn.g1_mul(opp.ped[2], int.from_bytes(bf, "big")))
    rp = zkat.RangeProof.deserialize(der_bytes)
    assert rp.serialize() == der_bytes
    assert zkat.rp_verify(V, opp.ped[1:], opp.left, opp.right, opp.P, opp.Q, opp.rounds, bits, rp) is None


def test_host_prover_out_of_range_rejected_by_oracle(host_pp, oracle_pp):
    """transfer_test.go:72-83: value 260 with an 8-bit PP -> invalid range proof"""
    pp = host_pp(8)
    opp = oracle_pp.with_bit_length(8)
    der_bytes, com = pp.prove_range(260, (5).to_bytes(32, "big"), seed=3)
    V = bn.g1_from_bytes(com)
    rp = zkat.RangeProof.deserialize(der_bytes)
    assert zkat.rp_verify(V, opp.ped[1:], opp.left, opp.right, opp.P, opp.Q, opp.rounds, 8, rp) == "invalid range proof"


def test_host_transfer_prover_accepted_by_oracle(host_pp, oracle_pp):
    pp = host_pp(8)
    opp = oracle_pp.with_bit_length(8)
    ib = [(11).to_bytes(32, "big"), (12).to_bytes(32, "big")]
    ob = [(13).to_bytes(32, "big"), (14).to_bytes(32, "big")]
    proof = pp.prove_transfer(b"ABC", [100, 50], ib, [120, 30], ob, seed=9)
    ins = [bn.g1_from_bytes(pp.token_commit(b"ABC", v, b)) for v, b in zip([100, 50], ib)]
    outs = [bn.g1_from_bytes(pp.token_commit(b"ABC", v, b)) for v, b in zip([120, 30], ob)]
    assert zkat.transfer_verify(opp, ins, outs, proof) == (None, -1)
    bad = pp.prove_transfer(b"ABC", [100, 50], ib, [120, 31], ob, seed=9)
    assert zkat.transfer_verify(opp, ins, outs, bad)[0] == "invalid transfer proof: invalid sum and type proof"


def test_host_issue_prover_accepted_by_oracle(host_pp, oracle_pp):
    pp = host_pp(8)
    opp = oracle_pp.with_bit_length(8)
    bfs = [(21).to_bytes(32, "big"), (22).to_bytes(32, "big")]
    proof = pp.prove_issue(b"XYZ", [7, 200], bfs, seed=4)
    toks = [bn.g1_from_bytes(pp.token_commit(b"XYZ", v, b)) for v, b in zip([7, 200], bfs)]
    assert zkat.issue_verify(opp, toks, proof) == (None, -1)


def test_shard_plan_contiguous_and_balanced():
    """fts_shard_plan: the split every multi-device entry point uses -- contiguous,
    covering [0, n), balanced by weight (caller order is preserved by construction)"""
    from fts_gpu import _lib as L
    assert L.shard_plan(10, 2) == [0, 5, 10]
    assert L.shard_plan(10, 3) == [0, 3, 7, 10]
    assert L.shard_plan(0, 4) == [0, 0, 0, 0, 0]
    assert L.shard_plan(3, 8)[-1] == 3 and len(L.shard_plan(3, 8)) == 9
    # issue-16 (weight 16.25) next to 2-in/2-out transfers (2.25): balanced by weight, not count
    w = [16.25] * 4 + [2.25] * 28
    b = L.shard_plan(len(w), 2, w)
    left, right = sum(w[:b[1]]), sum(w[b[1]:])
    assert b[0] == 0 and b[2] == len(w) and abs(left - right) <= 16.25
    import random
    rng = random.Random(3)
    for _ in range(50):
        n, k = rng.randrange(0, 200), rng.randrange(1, 9)
        w = [rng.choice([0.25, 2.25, 16.25]) for _ in range(n)]
        b = L.shard_plan(n, k, w)
        assert b[0] == 0 and b[-1] == n and all(x <= y for x, y in zip(b, b[1:]))
        tot = sum(w)
        for j in range(k):  # each shard within one item of its share
            assert abs(sum(w[b[j]:b[j + 1]]) - tot / k) <= 2 * 16.25 + 1e-9


def test_multi_device_context_merges_in_caller_order():
    """the merge side of the multi-device layer on CPU: shards write their verdicts
    at their offsets -- emulated over fts_shard_plan with a per-shard verifier"""
    from fts_gpu import _lib as L
    items = list(range(37))
    verdict = lambda x: (x * 7) % 5  # noqa: E731  (stand-in for a shard's device verdicts)
    for k in (1, 2, 3, 8):
        b = L.shard_plan(len(items), k)
        out = [None] * len(items)
        for j in range(k):
            lo, hi = b[j], b[j + 1]
            out[lo:hi] = [verdict(x) for x in items[lo:hi]]
        assert out == [verdict(x) for x in items]


def test_action_staging_host_only(host_pp):
    """fts_api.cpp act_stage on a host-only context (fts_debug_stage_actions): the
    chunked layout + direct-to-staging decode of transfers and issues, honest and
    malformed (truncated, empty, garbage, 1-in/1-out, nil sigma), more actions than
    one 128-action chunk -- no crash, FTS_API_OK, step timings filled"""
    import ctypes as C
    import random
    import fts_gpu
    from fts_gpu import _lib as L
    pp = host_pp(8)
    rng = random.Random(3)
    T = b"ABC"

    def bf():
        return rng.randrange(bn.R).to_bytes(32, "big")
    tr = []
    for i in range(6):
        n_in = 1 if i == 0 else 2
        n_out = 1 if i == 0 else 2
        iv = [rng.getrandbits(6) for _ in range(n_in)]
        ov = [sum(iv)] if n_out == 1 else [iv[0], iv[1]]
        ib, ob = [bf() for _ in iv], [bf() for _ in ov]
        ins = [pp.token_commit(T, v, x) for v, x in zip(iv, ib)]
        outs = [pp.token_commit(T, v, x) for v, x in zip(ov, ob)]
        tr.append((ins, outs, pp.prove_transfer(T, iv, ib, ov, ob, 77 + i)))
    ins, outs, p = tr[1]
    bad = [(ins, outs, p[:len(p) // 2]), (ins, outs, b""), (ins, outs, bytes(rng.getrandbits(8) for _ in range(300))),
           (ins, outs, p[:40] + b"\x00" * 20 + p[60:])]
    vals = [rng.getrandbits(8) for _ in range(3)]
    bfs = [bf() for _ in vals]
    iss = [([pp.token_commit(T, v, x) for v, x in zip(vals, bfs)], pp.prove_issue(T, vals, bfs, 99))]
    transfers = [(tr + bad)[i % (len(tr) + len(bad))] for i in range(300)]
    bt, bi = fts_gpu.TransferBatch(pp, transfers), fts_gpu.IssueBatch(pp, iss * 40)
    ms = (C.c_float * 4)()
    L.check("fts_debug_stage_actions", L.lib.fts_debug_stage_actions(pp._ctx, bt.n, bt.items, bi.n, bi.items, 2, ms))
    assert ms[0] > 0 and abs(ms[0] - (ms[1] + ms[2] + ms[3])) < 0.5 * ms[0] + 0.05
