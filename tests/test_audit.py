"""Token opening checks: Auditor.InspectOutput
(crypto/audit/auditor.go:226-238) and Token.ToClear (crypto/token/token.go:69-83)
re-commit HashToZr(type) ped0 + value ped1 + bf ped2 and compare it with
token.Data.

CPU tests pin the oracle (oracle.zkat.inspect_output) against the committed
fixtures (tests/golden/audit_golden.json, make_audit_golden.py) and the
library's host commitment; GPU tests run fts_token_open_batch and compare its
verdicts with the fixtures and with the oracle on seeded random batches."""
import json
import os
import random

import pytest

from conftest import GOLDEN

with open(os.path.join(GOLDEN, "audit_golden.json")) as f:
    CASES = json.load(f)


def _opening(c):
    h = lambda x: bytes.fromhex(x) if x is not None else None  # noqa: E731
    return (h(c["com"]), bytes.fromhex(c["type"]), h(c["value"]), h(c["bf"]))


def _want(F, expect):
    return {"ok": F.FTS_OK, "mismatch": F.FTS_E_OPEN_MISMATCH, "malformed": F.FTS_E_MALFORMED}[expect]


def test_oracle_matches_golden(oracle_pp):
    from oracle import zkat
    for c in CASES:
        err = zkat.inspect_output(oracle_pp.ped, *_opening(c))
        got = "ok" if err is None else ("malformed" if err == "malformed" else "mismatch")
        assert got == c["expect"], c["name"]
    assert {c["expect"] for c in CASES} == {"ok", "mismatch", "malformed"}


def test_host_commit_agrees_with_oracle(host_pp, oracle_pp):
    """the library's host commitment (fts_token_commit, token.go:208-217) == oracle"""
    from oracle import bn254 as bn, zkat
    rng = random.Random(5)
    for _ in range(4):
        v, bf = rng.randrange(2**64), rng.randrange(bn.R)
        t = b"T%d" % rng.randrange(9)
        assert host_pp(64).token_commit(t, v, bf.to_bytes(32, "big")) == \
            bn.g1_bytes(zkat.token_commit(oracle_pp.ped, t, v, bf))


def test_opening_batch_packing():
    """the fts_token_opening array points at the right bytes (nil fields -> NULL)"""
    import ctypes as C
    import fts_gpu
    ops = [_opening(c) for c in CASES]
    ob = fts_gpu.OpeningBatch(ops)
    for i, (com, t, v, bf) in enumerate(ops):
        it = ob.items[i]
        assert (C.string_at(it.com64, 64) if it.com64 else None) == com
        assert C.string_at(it.type, it.type_len) == t if it.type_len else t == b""
        assert (C.string_at(it.value32, 32) if it.value32 else None) == v
        assert (C.string_at(it.bf32, 32) if it.bf32 else None) == bf


def test_auditor_messages():
    import fts_gpu
    assert fts_gpu._inspect_message(fts_gpu.FTS_E_OPEN_MISMATCH, 2) == \
        "failed inspecting output [2]: output at index [2] does not match the provided opening"
    assert fts_gpu.L.status_str(fts_gpu.FTS_E_OPEN_MISMATCH) == "does not match the provided opening"


@pytest.mark.gpu
def test_gpu_openings_match_golden(gpu_pp):
    import fts_gpu as F
    pp = gpu_pp(64)
    st = pp.check_openings([_opening(c) for c in CASES])
    assert [int(s) for s in st] == [_want(F, c["expect"]) for c in CASES]


@pytest.mark.gpu
def test_gpu_openings_random_vs_oracle(gpu_pp, oracle_pp):
    """seeded random batch (honest, tampered value / bf / type, unreduced scalars) vs the oracle"""
    import fts_gpu as F
    from oracle import bn254 as bn, zkat
    rng = random.Random(0xA0D1)
    ops = []
    for i in range(96):
        t = b"TOK%d" % rng.randrange(5)
        v, bf = rng.randrange(2**64), rng.randrange(bn.R)
        com = bn.g1_bytes(zkat.token_commit(oracle_pp.ped, t, v, bf))
        m = i % 6
        if m == 1:
            v += 1
        elif m == 2:
            bf = (bf + 3) % bn.R
        elif m == 3:
            t += b"x"
        elif m == 4:
            v += bn.R  # unreduced: still the same commitment
        ops.append((com, t, v.to_bytes(32, "big"), bf.to_bytes(32, "big")))
    st = [int(s) for s in gpu_pp(64).check_openings(ops)]
    want = [F.FTS_OK if zkat.inspect_output(oracle_pp.ped, *o) is None else F.FTS_E_OPEN_MISMATCH for o in ops]
    assert st == want
    assert st.count(F.FTS_OK) == 48


@pytest.mark.gpu
def test_gpu_openings_large_batch_and_auditor(gpu_pp):
    """65,536 openings in one pass (tiled from a few distinct ones, the host
    commitment as producer); Auditor error chain on a tampered output"""
    import fts_gpu as F
    pp = gpu_pp(64)
    rng = random.Random(7)
    base = []
    for i in range(64):
        v, bf = rng.randrange(2**64), rng.randrange(2**250)
        t = b"ABC" if i % 2 else b"USD"
        base.append((pp.token_commit(t, v, bf.to_bytes(32, "big")), t, v.to_bytes(32, "big"), bf.to_bytes(32, "big")))
    ops = base * 1024
    bad = {5, 4097, 65535}
    for j in bad:
        com, t, v, bf = ops[j]
        ops[j] = (com, t, (int.from_bytes(v, "big") + 1).to_bytes(32, "big"), bf)
    st = pp.check_openings(ops)
    assert {int(i) for i in (st != F.FTS_OK).nonzero()[0]} == bad
    assert all(int(st[j]) == F.FTS_E_OPEN_MISMATCH for j in bad)
    aud = F.Auditor(pp)
    aud.InspectOutputs(base[:8])
    with pytest.raises(F.VerifyError) as e:
        aud.check_actions([base[:2], [base[2], ops[5]]], "tx1")
    assert str(e.value) == ("audit of 1 th transfer in tx [tx1] failed: failed inspecting output [1]: "
                            "output at index [1] does not match the provided opening")


def test_c_oracle_matches_golden(oracle_pp):
    """the C restatement (bench cpu_baseline) agrees with the fixtures (non-nil cases)"""
    from oracle import cref
    cases = [c for c in CASES if c["com"] is not None and c["value"] is not None and c["bf"] is not None]
    got = cref.open_check_many(oracle_pp, [_opening(c) for c in cases], threads=2)
    want = [{"ok": 0, "mismatch": 12, "malformed": 1}[c["expect"]] for c in cases]
    assert got == want


# ------------------------------------------- serialized metadata (token.go:136-158)
def _meta_cases():
    """(token.Data, driver.Metadata bytes, expected) built with fts_gpu.request's writer
    (token.Metadata.Serialize layout) from the golden openings"""
    from fts_gpu import request as rq
    out = []
    for c in CASES:
        com, t, v, bf = _opening(c)
        if com is None:
            continue
        try:
            t.decode("utf-8")
            expect = c["expect"]
        except UnicodeDecodeError:  # proto3 string field: invalid UTF-8 fails proto.Unmarshal
            expect = "malformed"
        out.append((c["name"], com, rq.token_metadata(t, v, bf), expect))
    com, t, v, bf = _opening(CASES[0])
    out += [("bad_typed_token_type", com, rq.token_metadata(t, v, bf, typ=3), "malformed"),
            ("nil_value", com, rq.token_metadata(t, None, bf), "malformed"),
            ("truncated", com, rq.token_metadata(t, v, bf)[:-5], "malformed"),
            ("short_element", com, rq.token_metadata(t, v.lstrip(b"\0"), bf), "ok"),
            ("issuer_set", com, rq.token_metadata(t, v, bf, issuer=b"alice"), "ok"),
            ("trailing_bytes", com, rq.token_metadata(t, v, bf) + b"\x00\x01", "ok")]
    return out


def test_metadata_decode_host():
    """fts_token_metadata_decode round-trips the writer; malformed forms are rejected"""
    import fts_gpu
    for name, com, meta, expect in _meta_cases():
        d = fts_gpu.decode_metadata(meta)
        if name in ("bad_typed_token_type", "truncated", "long_type"):
            assert d is None, name
            continue
        assert d is not None, name
        if name == "nil_value":
            assert d[1] is None
    c = next(c for c in CASES if c["name"] == "unreduced_value")
    com, t, v, bf = _opening(c)
    from oracle import bn254 as bn
    d = fts_gpu.decode_metadata(__import__("fts_gpu").request.token_metadata(t, v, bf))
    assert d[0] == t and int.from_bytes(d[1], "big") == int.from_bytes(v, "big") % bn.R and d[2] == bf


@pytest.mark.gpu
def test_gpu_metadata_openings(gpu_pp):
    import fts_gpu as F
    cases = _meta_cases()
    st = gpu_pp(64).check_metadata_openings([c[1] for c in cases], [c[2] for c in cases])
    assert [int(s) for s in st] == [_want(F, c[3]) for c in cases]
