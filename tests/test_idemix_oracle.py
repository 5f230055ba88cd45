"""Pins the idemix oracle (oracle/idemix.py) on the reference's own key fixtures
(tests/golden/idemix/: IssuerPublicKey / IssuerSecretKey files copied unchanged
from cmd/tokengen/testdata/idemix/ca, services/identity/idemix/testdata/
fp256bn_amcl/charlie.ExtraId2 and nogh/v1/validator/testdata/idemix/msp).

These pin BN254 HashToZr + Zr.Bytes (also used by every range-proof transcript
of the main path, oracle/bn254.py) and the idemix transcript encodings."""
import hashlib
import json
import os
import random

import pytest

from oracle import bn254, idemix

GOLD = os.path.join(os.path.dirname(__file__), "golden", "idemix")
FP256BN_P = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49F0CDC65FB12980A82D3292DDBAED33013
FP256BN_R = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49E0CDC65FB1299921AF62D536CD10B500D


def _raw(*p):
    with open(os.path.join(GOLD, *p), "rb") as f:
        return f.read()


@pytest.mark.parametrize("d", ["bn254_tokengen", "bn254_charlie"])
def test_bn254_ipk_hash_pins_hash_to_zr(d):
    raw = _raw(d, "IssuerPublicKey")
    ipk = idemix.parse_ipk(raw)
    body = idemix.ipk_hash_input(raw)
    assert len(body) == len(raw) - 34  # the hash field is last: 0x52 0x20 + 32 bytes
    assert idemix.zr_bytes(idemix.hash_to_zr(body)) == ipk["hash"]
    # the same HashToZr as the range-proof transcripts use
    assert bn254.hash_to_zr(body) == idemix.hash_to_zr(body)


def test_bn254_hash_to_zr_reduction_is_pinned():
    # the charlie key's SHA-256 digest exceeds r: the "mod r" step is observed
    raw = _raw("bn254_charlie", "IssuerPublicKey")
    dg = int.from_bytes(hashlib.sha256(idemix.ipk_hash_input(raw)).digest(), "big")
    assert dg >= bn254.R
    assert (dg % bn254.R).to_bytes(32, "big") == idemix.parse_ipk(raw)["hash"]


@pytest.mark.parametrize("d", ["fp256bn_validator", "fp256bn_crypto"])
def test_fp256bn_ipk_hash_and_curve(d):
    # the validator's and the crypto package's fixtures are FP256BN keys: same hash
    # rule mod that curve's order (two more independent HashToZr / Zr.Bytes pins)
    raw = _raw(d, "IssuerPublicKey")
    f = idemix.pb_fields(raw)
    h = [v for k, _, v in f if k == 10][0]
    dg = int.from_bytes(hashlib.sha256(idemix.ipk_hash_input(raw)).digest(), "big")
    assert (dg % FP256BN_R).to_bytes(32, "big") == h
    for k in (2, 3, 6, 7):  # h_sk, h_rand, bar_g1, bar_g2 on y^2 = x^3 + 3 over FP256BN
        e = dict((ff, v) for ff, _, v in idemix.pb_fields([v for kk, _, v in f if kk == k][0]))
        x, y = int.from_bytes(e[1], "big"), int.from_bytes(e[2], "big")
        assert (y * y - x ** 3 - 3) % FP256BN_P == 0


def test_bn254_issuer_key_proof_pins_encodings():
    for d in ("bn254_tokengen", "bn254_charlie"):
        ipk = idemix.parse_ipk(_raw(d, "IssuerPublicKey"))
        assert ipk["attribute_names"] == ["OU", "Role", "EnrollmentID", "RevocationHandle"]
        assert idemix.ipk_proof_valid(ipk)
        bad = dict(ipk, proof_s=(int.from_bytes(ipk["proof_s"], "big") + 1).to_bytes(32, "big"))
        assert not idemix.ipk_proof_valid(bad)


def test_fp256bn_nym_roundtrip_and_amcl_field_rules():
    ipk = idemix.parse_ipk(_raw("fp256bn_validator", "IssuerPublicKey"), idemix.FP256BNC)
    C = idemix.FP256BNC
    rng = random.Random(9)
    sk, rn = rng.randrange(C.r), rng.randrange(C.r)
    nym = idemix.make_nym(ipk, sk, rn)
    nb = C.g1_bytes(nym)
    assert len(nb) == 65 and nb[0] == 4
    sig = idemix.nym_sign(ipk, sk, nym, rn, b"msg", rng)
    idemix.nym_verify(ipk, nb, sig, b"msg")
    # AMCL FromBytes: bytes after the first 32 of a field are ignored; fewer than 32 panic
    f = idemix.pb_fields(sig)
    longer = b"".join(idemix.pb_bytes_field(k, v + b"\1" if k == 4 else v) for k, _, v in f)
    idemix.nym_verify(ipk, nb, longer, b"msg")
    short = b"".join(idemix.pb_bytes_field(k, v[1:] if k == 1 else v) for k, _, v in f)
    with pytest.raises(idemix.NymError, match="unmarshalling"):
        idemix.nym_verify(ipk, nb, short, b"msg")
    with pytest.raises(idemix.NymError, match="nym public key"):
        idemix.nym_verify(ipk, nb[1:], sig, b"msg")


def test_bn254_issuer_secret_key_relations():
    ipk = idemix.parse_ipk(_raw("bn254_tokengen", "IssuerPublicKey"))
    isk = int.from_bytes(_raw("bn254_tokengen", "IssuerSecretKey"), "big")
    assert bn254.g1_mul(ipk["bar_g1"], isk) == ipk["bar_g2"]
    assert idemix.g2_mul(ipk["w"], pow(isk, -1, bn254.R)) == idemix.G2_GEN


def test_nym_sign_verify_roundtrip_and_tampering():
    ipk = idemix.parse_ipk(_raw("bn254_tokengen", "IssuerPublicKey"))
    rng = random.Random(7)
    sk, rn = rng.randrange(bn254.R), rng.randrange(bn254.R)
    nym = idemix.make_nym(ipk, sk, rn)
    nb = bn254.g1_bytes(nym)
    msg = b"token request to sign" * 7
    sig = idemix.nym_sign(ipk, sk, nym, rn, msg, rng)
    idemix.nym_verify(ipk, nb, sig, msg)
    with pytest.raises(idemix.NymError, match="zero-knowledge proof is invalid"):
        idemix.nym_verify(ipk, nb, sig, msg + b"x")
    other = bn254.g1_bytes(idemix.make_nym(ipk, sk, rn + 1))
    with pytest.raises(idemix.NymError, match="zero-knowledge proof is invalid"):
        idemix.nym_verify(ipk, other, sig, msg)
    with pytest.raises(idemix.NymError, match="unmarshalling"):
        idemix.nym_verify(ipk, nb, b"", msg)
    with pytest.raises(idemix.NymError, match="unmarshalling"):
        idemix.nym_verify(ipk, nb, sig[:-3], msg)
    c, s1, s2, nonce = idemix.decode_nym_sig(sig)
    # an unreduced challenge fails Zr.Equals (integer comparison)
    with pytest.raises(idemix.NymError, match="zero-knowledge"):
        idemix.nym_verify(ipk, nb, idemix.encode_nym_sig(c + bn254.R, s1, s2, nonce), msg)
    # unreduced responses are used mod r (G1.Mul)
    idemix.nym_verify(ipk, nb, idemix.encode_nym_sig(c, s1 + bn254.R, s2, nonce), msg)


@pytest.mark.parametrize("curve", ["bn254", "fp256bn"])
def test_golden_nym_vectors(curve):
    """tests/golden/idemix_golden.json (tests/golden/make_idemix_golden.py) against the oracle."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "idemix_golden.json")) as f:
        g = json.load(f)[curve]
    C = idemix.BN254C if curve == "bn254" else idemix.FP256BNC
    assert g["curve"] == C.name
    ipk = idemix.parse_ipk(bytes.fromhex(g["ipk"]), C)
    for case in g["cases"]:
        want = case["error"]
        try:
            idemix.nym_verify(ipk, bytes.fromhex(case["nym"]), bytes.fromhex(case["sig"]), bytes.fromhex(case["msg"]))
            got = None
        except idemix.NymError as e:
            got = str(e)
        assert got == want, case["name"]


def test_issuer_key_fixtures_are_the_references():
    """the fixtures are the reference's files byte for byte (sha256 of the copies)"""
    want = {
        "bn254_tokengen": "701cea34637564a4921583877f4d19455f5a6cb28be8dc2023261637dea6569a",
        "bn254_charlie": "765568cad59f56ea169a8651b99e40bc4a2157700cdf9f06c3b13fd8412f8792",
        "fp256bn_validator": "74964ae62e43da2e41f12f43b1558317374748913f8dc4cb93d55a273141e1fa",
        "fp256bn_crypto": "bb1dc7f3d81ca64ce510e724743336b0307d6349440c7801de39ac3c9d32cb38",
    }
    for d, h in want.items():
        assert hashlib.sha256(_raw(d, "IssuerPublicKey")).hexdigest() == h, d


def test_fp256bn_crypto_key_digest_reduction():
    """nogh/v1/crypto's key: its SHA-256 digest exceeds BN254's r but not FP256BN's,
    so the stored hash also tells the two curves' reductions apart"""
    raw = _raw("fp256bn_crypto", "IssuerPublicKey")
    h = [v for k, _, v in idemix.pb_fields(raw) if k == 10][0]
    dg = int.from_bytes(hashlib.sha256(idemix.ipk_hash_input(raw)).digest(), "big")
    assert bn254.R <= dg < FP256BN_R
    assert (dg % bn254.R).to_bytes(32, "big") != h
    assert dg.to_bytes(32, "big") == h
