"""Pins the idemix identity oracle (oracle/pairing.py, oracle/pairing_tower.py,
oracle/idemix_identity.py) on the reference's own credential fixtures (CPU only).

tests/golden/idemix/ holds, copied unchanged (sha256 below):
* bn254_charlie/{IssuerPublicKey, SignerConfig}: services/identity/idemix/testdata/
  fp256bn_amcl/charlie.ExtraId2/{IssuerPublicKey, user/SignerConfig} (gurvy.Bn254)
* fp256bn_validator/{IssuerPublicKey, SignerConfig}: token/core/zkatdlog/nogh/v1/
  validator/testdata/idemix/{msp/IssuerPublicKey, user/SignerConfig} (FP256BN_AMCL)

Each SignerConfig carries a credential (A, B, E, S, attributes) issued under its
IssuerPublicKey, the user secret Sk, and a no-revocation CRI whose epoch key is
GenG2.  Credential.Ver's two equations hold on both curves:
  B == g1 + HRand*S + HSk*Sk + sum HAttrs[i]*attrs[i]
  e(W + g2*E, A) == e(g2, B)
which pins the curves, their G2 twists (BN254 D-type, FP256BN M-type), the G2
generators and encodings, the Credential proto layout and the pairing itself.
"""
import hashlib
import json
import os
import random

import pytest

from oracle import idemix as I, idemix_identity as ID, pairing as PR, pairing_tower as PT

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SHA = {
    ("bn254_charlie", "SignerConfig"): "c9c9c2a9b7dcbff4e4f55ca4cb20b34f4adf037850361539062b3b298128bdcf",
    ("fp256bn_validator", "SignerConfig"): "3f867d1679bd8198b01e8ff95cde0cae138db61e06f14affac5aed1c6e1c082f",
}
CURVES = {"bn254": ("bn254_charlie", I.BN254C, PR.BN254), "fp256bn": ("fp256bn_validator", I.FP256BNC, PR.FP256BN)}


def _raw(*p):
    with open(os.path.join(GOLD, "idemix", *p), "rb") as f:
        return f.read()


def _material(tag):
    d, C, PC = CURVES[tag]
    ipk_raw = _raw(d, "IssuerPublicKey")
    return ipk_raw, I.parse_ipk(ipk_raw, C), ID.parse_signer_config(_raw(d, "SignerConfig"), C), \
        ID.ipk_w(PC, ipk_raw), C, PC


def test_fixtures_unchanged():
    for (d, f), h in SHA.items():
        assert hashlib.sha256(_raw(d, f)).hexdigest() == h


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_credential_b_and_cri_generator(tag):
    ipk_raw, ipk, cred, W, C, PC = _material(tag)
    assert ipk["attribute_names"] == ["OU", "Role", "EnrollmentID", "RevocationHandle"]
    assert ID.credential_b(ipk, cred) == cred["B"]
    # the E / S order of the Credential proto is observable: swapped, B does not match
    assert ID.credential_b(ipk, dict(cred, S=cred["E"])) != cred["B"]
    # ALG_NO_REVOCATION: the CRI's epoch key is GenG2 (BN254: the standard gnark generator)
    assert ID.cri_epoch_pk(PC, cred["cri"]) == PC.g2_gen
    assert PC.g2_on_curve(W) and PC.g2_on_curve(PC.g2_gen)
    assert PC.g2_mul(PC.g2_gen, PC.r) is None  # order r


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_credential_pairing_pins_the_pairing(tag):
    _, ipk, cred, W, C, PC = _material(tag)
    assert ID.credential_pairing_ok(PC, W, cred)
    assert not ID.credential_pairing_ok(PC, W, dict(cred, E=cred["E"] + 1))
    assert not ID.credential_pairing_ok(PC, W, dict(cred, B=C.add(cred["B"], (1, 2))))


def test_fp256bn_twist_is_m_type():
    # the issuer's W is on y^2 = x^3 + 3(1 + i), not on the D-type twist y^2 = x^3 + 3/(1 + i)
    _, _, _, W, _, PC = _material("fp256bn")
    p = PC.p
    x, y = W
    rhs_d = PR.f2add(PR.f2mul(PR.f2mul(x, x, p), x, p), PR.f2mul((3, 0), PR.f2inv((1, 1), p), p), p)
    assert PR.f2mul(y, y, p) != rhs_d


@pytest.mark.parametrize("tag", ["bn254", "fp256bn"])
def test_device_algorithm_model_equals_direct_pairing(tag):
    """oracle/pairing_tower.py (the device's algorithm: precomputed lines, sparse
    line products, multi-Miller loop, u-chain final exponentiation) == the direct
    E(Fp12) pairing; bilinear"""
    _, _, _, W, C, PC = _material(tag)
    T = PT.Tower(PC)
    rng = random.Random(3)
    P = C.mul((1, 2), rng.randrange(1, C.r))
    assert T.to_poly(T.final_exp(T.miller([(T.lines(W), P)]))) == PC.pairing(W, P)
    a, b = rng.randrange(1, 1000), rng.randrange(1, 1000)
    lhs = T.final_exp(T.miller([(T.lines(PC.g2_mul(PC.g2_gen, a)), C.mul(P, b))]))
    base = T.final_exp(T.miller([(T.lines(PC.g2_gen), P)]))
    rhs = T.one()
    for bit in bin(a * b)[2:]:
        rhs = T.sq12(rhs)
        if bit == "1":
            rhs = T.m12(rhs, base)
    assert lhs == rhs


def test_pairing_constants_header_is_current():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert subprocess.call([sys.executable, os.path.join(root, "tools", "pairing_constants.py"), "--check"]) == 0


def test_golden_fixture_verdicts_reproduce():
    """a sample of the committed identity fixtures re-verified by the oracle (the
    fixture generator's verdicts are what the GPU tests compare with)"""
    with open(os.path.join(GOLD, "idemix_identity_golden.json")) as f:
        doc = json.load(f)
    for tag in ("bn254", "fp256bn"):
        _, ipk, _, W, C, PC = _material(tag)
        by = {c["name"]: c for c in doc[tag]["cases"]}
        for name in ("honest_0", "tampered_sE", "tampered_ABar", "no_rhnym", "nym_off_curve", "extra_ou_field"):
            c = by[name]
            try:
                ID.verify_identity(ipk, PC, W, bytes.fromhex(c["identity"]))
                got = None
            except ID.IdentityError as e:
                got = str(e)
            assert got == c["error"], name
        errs = [c["error"] for c in doc[tag]["cases"]]
        assert errs.count(None) >= 4 and len(set(errs)) >= 8


def test_bn254_g2_subgroup_check():
    """BN254 G2 decoding (oracle parse_ecp2) follows gnark-crypto's SetBytes: twist
    points outside the order-r subgroup are rejected; subgroup points, both issuer
    keys' W and the CRI epoch key (GenG2) decode; FP256BN (AMCL) has no such check"""
    C = PR.BN254
    for x in (7, 1234567, 99):
        q = ID.twist_point(C, x)
        assert C.g2_on_curve(q) and not ID.g2_in_subgroup(C, q)
        with pytest.raises(I.PointError):
            ID.parse_ecp2(C, ID.ecp2(C, q))
    for q in (C.g2_gen, C.g2_mul(C.g2_gen, 0xC0FFEE)):
        assert ID.parse_ecp2(C, ID.ecp2(C, q)) == q
    for tag in ("bn254", "fp256bn"):
        _, _, cred, W, _, PC = _material(tag)
        assert ID.g2_in_subgroup(PC, W) and ID.cri_epoch_pk(PC, cred["cri"]) == PC.g2_gen
    q = ID.twist_point(PR.FP256BN, 5)
    assert ID.parse_ecp2(PR.FP256BN, ID.ecp2(PR.FP256BN, q)) == q
