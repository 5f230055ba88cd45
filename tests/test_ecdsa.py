"""ECDSA P-256 owner signatures (the x509 half):
ecdsa.Verifier.Verify (validator/ecdsa/ecdsa.go:82-113).

CPU tests pin the oracle (oracle.ecdsa_p256) and the library's host-side
asn1/low-S parsing against tests/golden/ecdsa_golden.json — signatures made by
the OpenSSL CLI (make_ecdsa_golden.py), validity decided by
`openssl dgst -verify`, plus Go encoding/asn1 / IsLowS edge cases.  GPU tests
run fts_ecdsa_verify_batch through the C-ABI and compare every verdict with
the fixtures and with the oracle on seeded random batches."""
import json
import os
import random

import pytest

from conftest import GOLDEN

with open(os.path.join(GOLDEN, "ecdsa_golden.json")) as f:
    GOLD = json.load(f)["cases"]
# the X.x = r + n branch (make_ecdsa_crafted.py; validity double-checked with OpenSSL)
with open(os.path.join(GOLDEN, "ecdsa_crafted_golden.json")) as f:
    CRAFTED = json.load(f)["cases"]


def _case(c):
    pk = bytes.fromhex(c["pk64"])
    return bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"]), pk


def _pt(pk):
    return int.from_bytes(pk[:32], "big"), int.from_bytes(pk[32:], "big")


def _random_batch(n, seed, nkeys=8):
    from oracle import ecdsa_p256 as O
    rng = random.Random(seed)
    keys = []
    for _ in range(nkeys):
        d = rng.randrange(1, O.N)
        Q = O.mul(d, O.G)
        keys.append((d, Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")))
    msgs, sigs, pks = [], [], []
    for i in range(n):
        d, pk = keys[i % nkeys]
        m = rng.randbytes(rng.choice([0, 1, 55, 56, 63, 64, 65, 300, 2000]))
        sig = O.sign(d, m, rng.randrange(1, O.N))
        kind = i % 7
        if kind == 3:
            m = m + b"!"                      # tampered message
        elif kind == 5:
            r, s = O.parse_sig(sig)
            sig = O.der_sig(r, O.N - s)       # high-S twin
        msgs.append(m)
        sigs.append(sig)
        pks.append(pk)
    return msgs, sigs, pks


# ----------------------------------------------------------------------- CPU
def test_golden_has_openssl_cases():
    src = {c["src"] for c in GOLD}
    assert src == {"openssl", "rule"} and len(GOLD) >= 100
    assert {c["expect"] for c in GOLD} == {0, 13, 14, 15}


def test_oracle_matches_golden():
    from oracle import ecdsa_p256 as O
    for c in GOLD:
        m, s, pk = _case(c)
        assert O.verify(m, s, _pt(pk)) == c["expect"], c["tag"]


def test_oracle_matches_crafted_r_plus_n():
    from oracle import ecdsa_p256 as O
    assert [c["expect"] for c in CRAFTED] == [0, 15] * 3
    for c in CRAFTED:
        m, s, pk = _case(c)
        r, _ = O.parse_sig(s)
        assert O.verify(m, s, _pt(pk)) == c["expect"], c["tag"]
        assert (r < O.N) == (c["expect"] == 0)


def test_oracle_sign_roundtrip():
    from oracle import ecdsa_p256 as O
    msgs, sigs, pks = _random_batch(14, 7, nkeys=2)
    for i, (m, s, pk) in enumerate(zip(msgs, sigs, pks)):
        want = {3: O.SIG_INVALID, 5: O.SIG_NOT_LOW_S}.get(i % 7, O.OK)
        assert O.verify(m, s, _pt(pk)) == want


def test_host_parse_matches_golden():
    from fts_gpu import ecdsa as E
    from oracle import ecdsa_p256 as O
    for c in GOLD:
        _, sig, _ = _case(c)
        st, r, s = E.parse_sig(sig)
        if c["expect"] in (E.FTS_E_SIG_MALFORMED, E.FTS_E_SIG_NOT_LOW_S):
            assert st == c["expect"], c["tag"]
        elif c["expect"] == E.FTS_OK:
            assert st == E.FTS_OK and (r, s) == O.parse_sig(sig), c["tag"]
        else:
            assert st in (E.FTS_OK, E.FTS_E_SIG_INVALID), c["tag"]


def test_pkix_decode():
    import base64
    from fts_gpu import ecdsa as E
    from fts_gpu._lib import FtsError
    for c in GOLD[:8]:
        der = bytes.fromhex(c["pkix"])
        assert E.pk64_from_pkix(der) == bytes.fromhex(c["pk64"])
        pem = b"-----BEGIN PUBLIC KEY-----\n" + base64.encodebytes(der) + b"-----END PUBLIC KEY-----\n"
        assert E.pk64_from_pkix(pem) == bytes.fromhex(c["pk64"])
    with pytest.raises(FtsError):
        E.pk64_from_pkix(b"\x30" * 91)


def test_status_strings():
    from fts_gpu import ecdsa as E
    assert E.message(E.FTS_E_SIG_NOT_LOW_S) == "signature is not in lowS"
    assert E.message(E.FTS_E_SIG_INVALID) == "signature not valid"
    assert E.message(E.FTS_OK) is None


# ----------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_golden():
    from fts_gpu import ecdsa as E
    ms, ss, ps = zip(*[_case(c) for c in GOLD])
    st = E.verify_batch(ms, ss, ps, device=0)
    bad = [(c["tag"], int(s), c["expect"]) for c, s in zip(GOLD, st) if int(s) != c["expect"]]
    assert not bad, bad[:10]


@pytest.mark.gpu
def test_gpu_crafted_r_plus_n():
    """accept iff X.x == r or X.x == r + n (< p): the r + n branch is reached only by
    crafted signatures (ecdsa_kernels.hip final check)"""
    from fts_gpu import ecdsa as E
    ms, ss, ps = zip(*[_case(c) for c in CRAFTED])
    st = E.verify_batch(ms, ss, ps, device=0)
    assert [int(x) for x in st] == [c["expect"] for c in CRAFTED]


@pytest.mark.gpu
def test_gpu_random_vs_oracle():
    from fts_gpu import ecdsa as E
    from oracle import ecdsa_p256 as O
    msgs, sigs, pks = _random_batch(300, 0xEC0001)
    st = E.verify_batch(msgs, sigs, pks, device=0)
    want = [O.verify(m, s, _pt(p)) for m, s, p in zip(msgs, sigs, pks)]
    assert [int(x) for x in st] == want
    assert want.count(O.OK) > 150


@pytest.mark.gpu
def test_gpu_special_keys():
    """Q = G and Q = -G (u1*G and u2*Q land on the same subgroup line: the
    doubling / cancelling branches of the final addition)."""
    from fts_gpu import ecdsa as E
    from oracle import ecdsa_p256 as O
    rng = random.Random(5)
    msgs, sigs, pks = [], [], []
    for d in (1, 2, O.N - 1, O.N - 2):
        Q = O.mul(d, O.G)
        for _ in range(4):
            m = rng.randbytes(40)
            msgs.append(m)
            sigs.append(O.sign(d, m, rng.randrange(1, O.N)))
            pks.append(Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big"))
    st = E.verify_batch(msgs, sigs, pks)
    assert [int(x) for x in st] == [O.verify(m, s, _pt(p)) for m, s, p in zip(msgs, sigs, pks)]
    assert all(int(x) == 0 for x in st)


@pytest.mark.gpu
def test_gpu_large_tiled_batch():
    """Size-independent property at bench scale: a 40K batch tiled from 70
    oracle-checked signatures gives, item by item, the verdict of its source."""
    import numpy as np
    from fts_gpu import ecdsa as E
    from oracle import ecdsa_p256 as O
    msgs, sigs, pks = _random_batch(70, 0xEC0002)
    want = np.array([O.verify(m, s, _pt(p)) for m, s, p in zip(msgs, sigs, pks)], dtype=np.int32)
    n = 40000
    idx = np.arange(n) % 70
    st = E.verify_batch([msgs[i] for i in idx], [sigs[i] for i in idx], [pks[i] for i in idx])
    assert (st == want[idx]).all()
    t = E.last_timings(0)
    assert t["k_ecdsa_verify"] > 0


@pytest.mark.gpu
def test_gpu_verifier_api_and_empty():
    from fts_gpu import ecdsa as E
    c = next(c for c in GOLD if c["tag"] == "valid low-S")
    m, s, pk = _case(c)
    v = E.Verifier(bytes.fromhex(c["pkix"]))
    v.Verify(m, s)
    with pytest.raises(E.SignatureError, match="signature not valid"):
        v.Verify(m + b"x", s)
    hi = next(c for c in GOLD if c["tag"] == "valid high-S")
    with pytest.raises(E.SignatureError, match="signature is not in lowS"):
        E.Verifier(bytes.fromhex(hi["pk64"])).Verify(*_case(hi)[:2])
    assert len(E.verify_batch([], [], [])) == 0


def test_verify_packed_rejects_out_of_bounds():
    """bounds of the zero-copy form are checked before any pointer reaches the C library"""
    import numpy as np
    from fts_gpu import ecdsa as E
    m, s, pk = b"abcd", b"\x30" * 8, bytes(64)
    u = lambda *v: np.array(v, dtype=np.uint64)  # noqa: E731
    bad = [
        dict(msg_off=u(1), msg_len=u(4)),                       # message runs past its buffer
        dict(sig_off=u(0), sig_len=u(9)),                       # signature runs past its buffer
        dict(msg_off=u(2 ** 64 - 1), msg_len=u(2)),             # wrap-around offset
        dict(pk_buf=bytes(63)),                                 # short key buffer
        dict(msg_off=u(0, 0), msg_len=u(1, 1)),                 # unequal array lengths
    ]
    for kw in bad:
        args = dict(msg_buf=m, msg_off=u(0), msg_len=u(4), sig_buf=s, sig_off=u(0), sig_len=u(8), pk_buf=pk)
        args.update(kw)
        with pytest.raises(ValueError):
            E.verify_packed(**args)
