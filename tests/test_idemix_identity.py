"""GPU: idemix identity validity (fts_idemix_identity_verify_batch) against the
oracle's verdicts on identities built from the reference's own credentials
(tests/golden/idemix_identity_golden.json, tests/golden/make_idemix_identity_golden.py),
on both curves: golden cases (honest, tampered responses / points, missing
EidNym / RhNym, revocation, malformed protos and keys), the device pairing
against the oracle's GT value, wrong-issuer identities, and a 65,536-identity
batch at exact positions."""
import json
import os
import random

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def _doc():
    with open(os.path.join(GOLD, "idemix_identity_golden.json")) as f:
        return json.load(f)


def _ipk(d):
    with open(os.path.join(GOLD, "idemix", d, "IssuerPublicKey"), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def verifiers():
    from fts_gpu import idemix as I
    doc = _doc()
    vs = {tag: I.IdentityVerifier(_ipk(doc[tag]["issuer"]), device=0, curve=doc[tag]["curve_id"])
          for tag in ("bn254", "fp256bn")}
    yield vs
    for v in vs.values():
        v.close()


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_golden_identity_verdicts(verifiers, tag):
    from fts_gpu import idemix as I
    cases = _doc()[tag]["cases"]
    st = verifiers[tag].verify_batch([bytes.fromhex(c["identity"]) for c in cases])
    got = {c["name"]: I.message(int(s)) for c, s in zip(cases, st)}
    want = {c["name"]: c["error"] for c in cases}
    assert got == want


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_single_identity_api(verifiers, tag):
    from fts_gpu import idemix as I
    by = {c["name"]: c for c in _doc()[tag]["cases"]}
    verifiers[tag].Deserialize(bytes.fromhex(by["honest_1"]["identity"]))
    with pytest.raises(I.IdentityError, match="zero-knowledge proof is invalid"):
        verifiers[tag].Deserialize(bytes.fromhex(by["tampered_sE"]["identity"]))
    assert len(verifiers[tag].verify_batch([])) == 0


def test_device_pairing_equals_oracle_gt(verifiers):
    """e(W, P) and e(g2, P) from the device (after the final exponentiation) equal
    the oracle's optimal ate values coefficient for coefficient (BN254)"""
    from oracle import idemix as OI, idemix_identity as ID, pairing as PR, pairing_tower as PT
    PC, C = PR.BN254, OI.BN254C
    T = PT.Tower(PC)
    W = ID.ipk_w(PC, _ipk("bn254_charlie"))
    P = C.mul((1, 2), 123456789)
    R = 1 << 256
    for which, Q in ((0, W), (1, PC.g2_gen)):
        dev = verifiers["bn254"].pairing_debug(which, C.g1_bytes(P))
        want = T._zs(T.final_exp(T.miller([(T.lines(Q), P)])))
        got = [((a * pow(R, -1, PC.p)) % PC.p, (b * pow(R, -1, PC.p)) % PC.p) for a, b in dev]
        assert got == [tuple(z) for z in want], which
        # Miller value too (before the final exponentiation): same algorithm step for step
        devm = verifiers["bn254"].pairing_debug(which, C.g1_bytes(P), final_exp=False)
        wantm = T._zs(T.miller([(T.lines(Q), P)]))
        gotm = [((a * pow(R, -1, PC.p)) % PC.p, (b * pow(R, -1, PC.p)) % PC.p) for a, b in devm]
        assert gotm == [tuple(z) for z in wantm], which


def test_wrong_issuer_rejected():
    """charlie's BN254 identities under the tokengen BN254 issuer key: the pairing
    (or the transcript, which hashes ipk.Hash) fails"""
    from fts_gpu import idemix as I
    doc = _doc()
    with open(os.path.join(GOLD, "idemix", "bn254_tokengen", "IssuerPublicKey"), "rb") as f:
        other = I.IdentityVerifier(f.read(), device=0, curve=I.FTS_CURVE_BN254)
    ids = [bytes.fromhex(c["identity"]) for c in doc["bn254"]["cases"] if c["name"].startswith("honest")]
    st = other.verify_batch(ids)
    other.close()
    assert all(int(s) == I.FTS_E_ID_PAIRING for s in st)


def test_bad_issuer_keys_rejected():
    from fts_gpu import idemix as I
    from fts_gpu import _lib as L
    with pytest.raises(L.FtsError):
        I.IdentityVerifier(_ipk("bn254_charlie")[:200], device=0, curve=I.FTS_CURVE_BN254)
    with pytest.raises(L.FtsError):  # a BN254 key read as FP256BN: points off that curve
        I.IdentityVerifier(_ipk("bn254_charlie"), device=0, curve=I.FTS_CURVE_FP256BN_AMCL)


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_large_batch_exact_positions(verifiers, tag):
    """65,536 identities (the fixture tile of 64, 1 in 8 tampered, repeated and
    shuffled with golden cases mixed in): every verdict at its position"""
    from fts_gpu import idemix as I
    doc = _doc()[tag]
    pool = [(bytes.fromhex(t["identity"]), t["error"]) for t in doc["tile"]]
    pool += [(bytes.fromhex(c["identity"]), c["error"]) for c in doc["cases"]]
    rng = random.Random(7)
    n = 65536
    pick = [rng.randrange(len(pool)) for _ in range(n)]
    st = verifiers[tag].verify_batch([pool[k][0] for k in pick])
    want = np.array([pool[k][1] is None for k in pick])
    assert ((st == 0) == want).all()
    msgs = {k: I.message(int(s)) for k, s in zip(pick[:4096], st[:4096])}
    assert all(msgs[k] == pool[k][1] for k in msgs)
    t = verifiers[tag].last_kernel_ms()
    assert t[0] > 0 and t[1] > 0


def _key(f, wt):
    k, out = (f << 3) | wt, b""
    while True:
        c = k & 0x7F
        k >>= 7
        out += bytes([c | (0x80 if k else 0)])
        if not k:
            return out


def _overlong(f, wt, last):
    """the key of (f, wt) as a 10-byte varint whose last byte is `last`"""
    k = (f << 3) | wt
    body = [(k >> (7 * i)) & 0x7F for i in range(9)]
    return bytes(b | 0x80 for b in body) + bytes([last])


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_identity_proto_wire_edge_cases(verifiers, tag):
    """protowire semantics of the SerializedIdemixIdentity reader (host/pb.hpp):
    a 10-byte key varint is accepted when its last byte is 0 or 1 and rejected as an
    overflow above (protowire.ConsumeVarint); an unknown group field is skipped
    (ConsumeFieldValue), a group without its end is malformed"""
    from fts_gpu import idemix as I
    from oracle import idemix as OI
    by = {c["name"]: c for c in _doc()[tag]["cases"]}
    raw = bytes.fromhex(by["honest_1"]["identity"])
    fields = OI.pb_fields(raw)
    rebuilt = b"".join(OI.pb_bytes_field(f, v) for f, wt, v in fields)
    assert rebuilt == raw and all(wt == 2 for _, wt, _ in fields)

    def with_key(i, key):
        out = b""
        for j, (f, wt, v) in enumerate(fields):
            enc = OI.pb_bytes_field(f, v)
            out += (key + enc[len(_key(f, 2)):]) if j == i else enc
        return out
    group = _key(100, 3) + _key(1, 0) + b"\x05" + _key(2, 2) + b"\x01Z" + _key(100, 4)
    cases = [
        (with_key(0, _overlong(fields[0][0], 2, 0x00)), 0),                        # overlong, no overflow
        (with_key(0, _overlong(fields[0][0], 2, 0x02)), I.FTS_E_ID_MALFORMED),     # 10th byte > 1: overflow
        (with_key(len(fields) - 1, _overlong(fields[-1][0], 2, 0x7F)), I.FTS_E_ID_MALFORMED),
        (raw + group, 0),                                                          # unknown group skipped
        (group + raw, 0),
        (raw + _key(100, 3) + _key(1, 0) + b"\x05", I.FTS_E_ID_MALFORMED),         # group without its end
        (raw + _key(100, 3) + _key(101, 4), I.FTS_E_ID_MALFORMED),                 # mismatched end group
        (raw + _key(100, 4), I.FTS_E_ID_MALFORMED),                                # end group alone
    ]
    st = verifiers[tag].verify_batch([c for c, _ in cases])
    assert [int(s) for s in st] == [w for _, w in cases]
    # the oracle's wire reader agrees on which encodings parse
    for c, w in cases:
        try:
            OI.pb_fields(c)
            ok = True
        except ValueError:
            ok = False
        assert ok == (w == 0), c.hex()[:40]


def _with_epoch_key(raw, key_proto):
    """an identity whose Signature carries another revocation epoch key (field 14);
    the key is not in the proof's transcript, so only its decoding decides"""
    from oracle import idemix as OI, idemix_identity as ID
    outer = OI.pb_fields(raw)
    out = b""
    for f, wt, v in outer:
        if f == 4:
            sig = b""
            for sf, swt, sv in OI.pb_fields(v):
                if sf == 14:
                    sv = key_proto
                sig += OI.pb_bytes_field(sf, sv) if swt == 2 else ID._varint_field(sf, sv)
            v = sig
        out += OI.pb_bytes_field(f, v)
    return out


def test_bn254_g2_subgroup_checks(verifiers):
    """gnark-crypto's G2Affine.SetBytes (mathlib NewG2FromBytes, BN254) rejects twist
    points outside the order-r subgroup: an epoch key on the twist but off the
    subgroup makes the identity malformed, a subgroup key does not;
    distinct keys in one batch are each checked once (host dedupe) and once per
    context (verdict cache), every verdict at its position; an issuer key whose W is
    off the subgroup is refused"""
    from fts_gpu import idemix as I
    from fts_gpu import _lib as L
    from oracle import idemix as OI, idemix_identity as ID, pairing as PR
    C = PR.BN254
    by = {c["name"]: c for c in _doc()["bn254"]["cases"]}
    honest = bytes.fromhex(by["honest_1"]["identity"])
    bad = [ID.twist_point(C, x) for x in (7, 1234567)]
    assert all(C.g2_on_curve(q) and not ID.g2_in_subgroup(C, q) for q in bad)
    good = [C.g2_gen, C.g2_add(C.g2_gen, C.g2_gen), C.g2_mul(C.g2_gen, 0xC0FFEE)]
    keys = [(ID.ecp2(C, q), 0) for q in good] + [(ID.ecp2(C, q), I.FTS_E_ID_MALFORMED) for q in bad]
    ids = [(_with_epoch_key(honest, k), w) for k, w in keys]
    st = verifiers["bn254"].verify_batch([x for x, _ in ids])
    assert [int(s) for s in st] == [w for _, w in ids]
    # the context caches each distinct key's verdict: a second batch mixes cached
    # keys with ones it has not seen (a third off-subgroup point, a new subgroup
    # point), every verdict at its position, and a third call hits only the cache
    more = [(ID.ecp2(C, ID.twist_point(C, 99)), I.FTS_E_ID_MALFORMED), (ID.ecp2(C, C.g2_mul(C.g2_gen, 77)), 0)]
    assert not ID.g2_in_subgroup(C, ID.twist_point(C, 99))
    ids += [(_with_epoch_key(honest, k), w) for k, w in more]
    rng = random.Random(11)
    for _ in range(2):
        pick = [rng.randrange(len(ids)) for _ in range(2000)]
        st = verifiers["bn254"].verify_batch([ids[k][0] for k in pick])
        assert [int(s) for s in st] == [ids[k][1] for k in pick]
    # issuer key with W off the subgroup (field 5 of IssuerPublicKey)
    ipk = _ipk("bn254_charlie")
    fields = OI.pb_fields(ipk)
    w_bad = b"".join(OI.pb_bytes_field(f, ID.ecp2(C, bad[0]) if f == 5 else v) if wt == 2 else ID._varint_field(f, v)
                     for f, wt, v in fields)
    with pytest.raises(L.FtsError):
        I.IdentityVerifier(w_bad, device=0, curve=I.FTS_CURVE_BN254)


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_batch_pairing_check_groups(verifiers, tag, monkeypatch):
    """the randomised group pairing check (k_idv_bp_*): a batch whose identities all
    satisfy the pairing equation (honest and ZK-tampered ones) pairs no identity one
    by one; identities failing the equation ("APrime and ABar don't have the expected
    structure") at known positions send exactly their groups of 256 to the one-by-one
    pairing, and every verdict at its position equals the per-identity path's
    (FTS_IDV_BATCH=0)"""
    from fts_gpu import idemix as I
    doc = _doc()[tag]
    V = verifiers[tag]
    tile = [(bytes.fromhex(t["identity"]), t["error"]) for t in doc["tile"]]
    n = 8192
    ids = [tile[(7 * i) % len(tile)] for i in range(n)]
    st = V.verify_batch([x for x, _ in ids])
    assert [I.message(int(s)) for s in st] == [e for _, e in ids]
    assert V.last_pairing_stats() == (n // 256, 0)
    # pairing failures in groups 3 and 17 (two in group 17)
    bad = [c for c in doc["cases"] if c["error"] == "signature invalid: APrime and ABar don't have the expected structure"]
    assert bad
    pos = [3 * 256 + 5, 17 * 256 + 100, 17 * 256 + 255]
    for j, p in enumerate(pos):
        ids[p] = (bytes.fromhex(bad[j % len(bad)]["identity"]), bad[j % len(bad)]["error"])
    st = V.verify_batch([x for x, _ in ids])
    assert [I.message(int(s)) for s in st] == [e for _, e in ids]
    groups, paired = V.last_pairing_stats()
    assert groups == n // 256 and paired == 2 * 256  # every identity of the two groups decodes
    # the per-identity path agrees verdict for verdict
    monkeypatch.setenv("FTS_IDV_BATCH", "0")
    W = I.IdentityVerifier(_ipk(doc["issuer"]), device=0, curve=doc["curve_id"])
    try:
        st0 = W.verify_batch([x for x, _ in ids])
        assert W.last_pairing_stats() == (0, n)
    finally:
        W.close()
    assert (st0 == st).all()


def test_batch_pairing_check_wrong_issuer():
    """every group fails under another issuer's W: all identities are paired one by one"""
    from fts_gpu import idemix as I
    doc = _doc()
    with open(os.path.join(GOLD, "idemix", "bn254_tokengen", "IssuerPublicKey"), "rb") as f:
        other = I.IdentityVerifier(f.read(), device=0, curve=I.FTS_CURVE_BN254)
    ids = [bytes.fromhex(t["identity"]) for t in doc["bn254"]["tile"]] * 8
    try:
        st = other.verify_batch(ids)
        assert all(int(s) == I.FTS_E_ID_PAIRING for s in st)
        assert other.last_pairing_stats() == (2, len(ids))
    finally:
        other.close()
