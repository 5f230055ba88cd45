"""Idemix identity validity (the association proof of a serialized idemix owner
identity), restated in pure Python.  ORACLE / TEST INFRASTRUCTURE ONLY: never
imported by the product path.

Reference call chain (fabric-token-sdk), run for EVERY transfer input with no
cache:
* validator/validator_transfer.go:46  ctx.Deserializer.GetOwnerVerifier(tok.Owner)
* core/common/deserializer.go:63-64   d.ownerDeserializer.DeserializeVerifier(id)
* services/identity/idemix/deserializer.go:82-93  i.Deserialize(raw, true)
  (verification type ExpectEidNymRhNym, deserializer.go:35; no revocation key,
  epoch 0, no NymEID metadata)
* services/identity/idemix/crypto/deserializer.go:36-86  proto.Unmarshal of
  SerializedIdemixIdentity (crypto/protos/idemix_config.proto: 1 nym_public_key,
  4 proof), empty nym rejected, nym KeyImport, then id.Validate()
* services/identity/idemix/crypto/id.go:74-108  verifyProof -> CSP.Verify(ipk,
  proof, nil, IdemixSignerOpts{4 hidden attributes, RhIndex 3, EidIndex 2})
  -> IBM/idemix Signature.Ver (github.com/IBM/idemix
  v0.0.2-0.20240816143710-3dce4618d760, bccsp/schemes/dlog/crypto/signature.go;
  NOT vendored: restated from the published code).

Signature.Ver, as restated (all attributes hidden, no message):
  pairing   APrime != O and e(W, APrime) == e(g2, ABar)
  t1 = APrime*sE + HRand*sR2 - (ABar - BPrime)*c
  t2 = HRand*sS' + BPrime*sR3 + HSk*sSk + sum_i HAttrs[i]*sAttrs[i] + g1*c
  t3 = HSk*sSk + HRand*sRNym - Nym*c
  t4 = HAttrs[2]*sAttrs[2] + HRand*sEid - EidNym*c       (ExpectEidNymRhNym)
  t5 = HAttrs[3]*sAttrs[3] + HRand*sRh - RhNym*c
  c' = HashToZr("signWithEidNymRhNym" || t1 || t2 || t3 || APrime || ABar ||
                BPrime || Nym || EidNym || t4 || RhNym || t5 || ipk.Hash ||
                Disclosure(4 zero bytes))
  accept iff c == HashToZr(c' || Nonce)

PINNED by the reference's own fixtures (tests/test_idemix_identity_oracle.py):
the pairing on both curves, the G2 generators and encodings, the Credential proto
(A, B, E, S, attributes), g1, and B = g1 + HRand*S + HSk*sk + sum HAttrs*attrs,
through the two SignerConfig credentials (oracle/pairing.py); HashToZr, Zr.Bytes
and the G1 encodings through the IssuerPublicKey fixtures (oracle/idemix.py).
UNPINNED (no identity-proof vector exists in the reference): the Signature proto
field numbers, the label, the order of the t-values and nyms in the transcript,
the response signs, the EidNym/RhNym sub-proofs and the error precedence; and
that the proof's Nym is not compared with the identity's nym_public_key (the
restated Ver never reads the latter).
"""
from . import idemix as I
from . import pairing as PR

LABEL = b"signWithEidNymRhNym"
EID_INDEX, RH_INDEX = 2, 3
N_ATTRS = 4

# error classes (fts_status numbering of the library, FTS_E_ID_*)
E_ID_MALFORMED = "identity malformed"                 # proto / empty nym / point encodings
E_ID_BADNYM = "failed to import nym public key"
E_ID_NO_EIDNYM = "no EidNym provided but ExpectEidNym required"
E_ID_NO_RHNYM = "no RhNym provided but ExpectEidNymRhNym required"
E_ID_REVOCATION = "unsupported revocation algorithm"
E_ID_APRIME = "signature invalid: APrime = 1"
E_ID_PAIRING = "signature invalid: APrime and ABar don't have the expected structure"
E_ID_ZK = "signature invalid: zero-knowledge proof is invalid"

CURVE_PAIRING = {id(I.BN254C): PR.BN254, id(I.FP256BNC): PR.FP256BN}


class IdentityError(ValueError):
    pass


# ------------------------------------------------------------- encodings
def ecp(pt):
    """G1 -> idemix ECP proto {1 x, 2 y} (32-byte big-endian coordinates)"""
    return I.pb_bytes_field(1, pt[0].to_bytes(32, "big")) + I.pb_bytes_field(2, pt[1].to_bytes(32, "big"))


def ecp2(curve_pr, Q):
    """G2 -> ECP2 proto {1 xa, 2 xb, 3 ya, 4 yb}: gnark raw order (imaginary part
    first) for BN254, AMCL (real part first) for FP256BN"""
    (x0, x1), (y0, y1) = Q
    vals = (x1, x0, y1, y0) if curve_pr is PR.BN254 else (x0, x1, y0, y1)
    return b"".join(I.pb_bytes_field(i + 1, v.to_bytes(32, "big")) for i, v in enumerate(vals))


def parse_ecp2(curve_pr, raw):
    f = I.pb_fields(raw)
    parts = [I._pb_bytes(f, i) for i in (1, 2, 3, 4)]
    if any(len(p) != 32 for p in parts):
        raise I.PointError("ECP2 coordinate length")
    v = [int.from_bytes(p, "big") for p in parts]
    if max(v) >= curve_pr.p:
        raise I.PointError("non-canonical G2 coordinate")
    Q = ((v[1], v[0]), (v[3], v[2])) if curve_pr is PR.BN254 else ((v[0], v[1]), (v[2], v[3]))
    if Q == ((0, 0), (0, 0)):
        return None
    if not curve_pr.g2_on_curve(Q):
        raise I.PointError("G2 point not on curve")
    if curve_pr is PR.BN254 and not g2_in_subgroup(curve_pr, Q):
        # gnark-crypto G2Affine.SetBytes (mathlib NewG2FromBytes) checks the subgroup;
        # AMCL's ECP2_fromBytes (FP256BN) does not
        raise I.PointError("G2 point not in the r-torsion subgroup")
    return Q


def twist_point(curve_pr, x0):
    """a point of the twist y^2 = x^3 + b' with x = (x0 + k, 1) for the first k that
    gives a square (any subgroup: the test vectors' off-subgroup points); p = 3 mod 4
    square root in Fp2 = Fp[u]/(u^2 + 1) (Adj / Rodriguez-Henriquez, algorithm 9)"""
    p = curve_pr.p
    assert p % 4 == 3

    def f2pow(a, e):
        r = (1, 0)
        while e:
            if e & 1:
                r = PR.f2mul(r, a, p)
            a = PR.f2mul(a, a, p)
            e >>= 1
        return r
    k = 0
    while True:
        x = ((x0 + k) % p, 1)
        a = PR.f2add(PR.f2mul(PR.f2mul(x, x, p), x, p), curve_pr.b2, p)
        a1 = f2pow(a, (p - 3) // 4)
        alpha = PR.f2mul(PR.f2mul(a1, a1, p), a, p)
        a0 = PR.f2mul((alpha[0], (-alpha[1]) % p), alpha, p)  # alpha^p * alpha
        if a0 != (p - 1, 0):
            x_0 = PR.f2mul(a1, a, p)
            if alpha == (p - 1, 0):
                y = PR.f2mul((0, 1), x_0, p)
            else:
                y = PR.f2mul(f2pow(PR.f2add((1, 0), alpha, p), (p - 1) // 2), x_0, p)
            if PR.f2mul(y, y, p) == a:
                return (x, y)
        k += 1


def g2_in_subgroup(curve_pr, Q):
    """[r] Q == O, by double-and-add without reducing the scalar mod r"""
    acc = None
    for bit in bin(curve_pr.r)[2:]:
        acc = curve_pr.g2_add(acc, acc)
        if bit == "1":
            acc = curve_pr.g2_add(acc, Q)
    return acc is None


def _varint_field(f, v):
    out, k = b"", (f << 3)
    while True:
        c = k & 0x7F
        k >>= 7
        out += bytes([c | (0x80 if k else 0)])
        if not k:
            break
    while True:
        c = v & 0x7F
        v >>= 7
        out += bytes([c | (0x80 if v else 0)])
        if not v:
            return out


def encode_signature(s, curve_pr):
    """idemix Signature proto (field numbers restated, unpinned)"""
    zb = I.zr_bytes
    out = I.pb_bytes_field(1, ecp(s["APrime"])) + I.pb_bytes_field(2, ecp(s["ABar"])) + \
        I.pb_bytes_field(3, ecp(s["BPrime"]))
    for f, k in ((4, "c"), (5, "sSk"), (6, "sE"), (7, "sR2"), (8, "sR3"), (9, "sSPrime")):
        out += I.pb_bytes_field(f, zb(s[k]))
    for a in s["sAttrs"]:
        out += I.pb_bytes_field(10, zb(a))
    out += I.pb_bytes_field(11, zb(s["nonce"])) + I.pb_bytes_field(12, ecp(s["Nym"])) + \
        I.pb_bytes_field(13, zb(s["sRNym"]))
    if s.get("epoch_pk", 0) is not None:
        out += I.pb_bytes_field(14, ecp2(curve_pr, s.get("epoch_pk") or curve_pr.g2_gen))
    if s.get("epoch"):
        out += _varint_field(16, s["epoch"])
    nr = b"" if not s.get("rev_alg") else _varint_field(1, s["rev_alg"])
    out += I.pb_bytes_field(17, nr)
    if s.get("EidNym") is not None:
        out += I.pb_bytes_field(18, I.pb_bytes_field(1, ecp(s["EidNym"])) + I.pb_bytes_field(2, zb(s["sEid"])))
    if s.get("RhNym") is not None:
        out += I.pb_bytes_field(19, I.pb_bytes_field(1, ecp(s["RhNym"])) + I.pb_bytes_field(2, zb(s["sRh"])))
    return out


def serialize_identity(nym_bytes, proof):
    return I.serialize_identity(nym_bytes, proof=proof)


# ---------------------------------------------------------- credentials
def parse_signer_config(raw, curve):
    """IdemixSignerConfig (proto, or the JSON form idemixgen writes with base64
    fields) -> credential parts and the user secret"""
    import base64
    import json
    try:
        j = json.loads(raw)
        cred, sk = base64.b64decode(j["Cred"]), base64.b64decode(j["Sk"])
        cri = base64.b64decode(j.get("credential_revocation_information", ""))
        eid = j.get("enrollment_id", "").encode()
    except (ValueError, UnicodeDecodeError):
        f = I.pb_fields(raw)
        cred, sk, cri, eid = (I._pb_bytes(f, 1), I._pb_bytes(f, 2), I._pb_bytes(f, 6), I._pb_bytes(f, 5))
    f = I.pb_fields(cred)
    return {
        "A": I._ecp(I._pb_bytes(f, 1), curve), "B": I._ecp(I._pb_bytes(f, 2), curve),
        "E": int.from_bytes(I._pb_bytes(f, 3), "big"), "S": int.from_bytes(I._pb_bytes(f, 4), "big"),
        "attrs": [int.from_bytes(v, "big") for k, _, v in f if k == 5],
        "sk": int.from_bytes(sk, "big"), "cri": cri, "enrollment_id": eid,
    }


def cri_epoch_pk(curve_pr, cri):
    """CredentialRevocationInformation.epoch_pk (field 2): for ALG_NO_REVOCATION
    idemix writes GenG2 there"""
    return parse_ecp2(curve_pr, I._pb_bytes(I.pb_fields(cri), 2))


def ipk_w(curve_pr, ipk_raw):
    return parse_ecp2(curve_pr, I._pb_bytes(I.pb_fields(ipk_raw), 5))


def credential_b(ipk, cred):
    """g1 + HRand*S + HSk*sk + sum HAttrs[i]*attrs[i] (Credential.Ver's B check)"""
    C = ipk["curve"]
    acc = C.add((1, 2), C.add(C.mul(ipk["h_rand"], cred["S"]), C.mul(ipk["h_sk"], cred["sk"])))
    for h, a in zip(ipk["h_attrs"], cred["attrs"]):
        acc = C.add(acc, C.mul(h, a))
    return acc


def credential_pairing_ok(curve_pr, W, cred):
    """e(W + g2*E, A) * e(-g2, B) == 1"""
    Q = curve_pr.g2_add(W, curve_pr.g2_mul(curve_pr.g2_gen, cred["E"]))
    return curve_pr.pairing_product_is_one([(Q, cred["A"]), (curve_pr.g2_neg(curve_pr.g2_gen), cred["B"])])


# ------------------------------------------------------------- transcript
def _challenge(C, ipk_hash, pts, nonce):
    data = LABEL + b"".join(C.g1_bytes(p) for p in pts) + ipk_hash[:32].ljust(32, b"\0") + bytes(N_ATTRS)
    c1 = C.hash_to_zr(data)
    return C.hash_to_zr(I.zr_bytes(c1) + I.zr_bytes(nonce)), data


def sign(ipk, cred, nym_sk_rand, rng, curve_pr, rev_alg=0, epoch=0, drop=()):
    """NewSignature(cred, sk, Nym, RNym, ipk, Disclosure 0000, msg nil, rhIndex 3,
    eidIndex 2, CRI, EidNymRhNym) with randomness from `rng` (random.Random;
    fixtures only).  Returns (signature dict, Nym point).  `drop` omits EidNym /
    RhNym for negative cases."""
    C = ipk["curve"]
    r = C.r
    R = lambda: rng.randrange(1, r)  # noqa: E731
    sk, rnym = cred["sk"], nym_sk_rand
    Nym = C.add(C.mul(ipk["h_sk"], sk), C.mul(ipk["h_rand"], rnym))
    r1, r2 = R(), R()
    r3 = pow(r1, r - 2, r)
    nonce = R()
    A, B, E, S = cred["A"], cred["B"], cred["E"], cred["S"]
    APrime = C.mul(A, r1)
    ABar = C.add(C.mul(B, r1), C.neg(C.mul(APrime, E)))
    BPrime = C.add(C.mul(B, r1), C.neg(C.mul(ipk["h_rand"], r2)))
    sPrime = (S - r2 * r3) % r
    rSk, re, rR2, rR3, rSP, rRNym = (R() for _ in range(6))
    rAttrs = [R() for _ in range(N_ATTRS)]
    t1 = C.add(C.mul(APrime, re), C.mul(ipk["h_rand"], rR2))
    t2 = C.add(C.mul(ipk["h_rand"], rSP), C.add(C.mul(BPrime, rR3), C.mul(ipk["h_sk"], rSk)))
    for h, ra in zip(ipk["h_attrs"], rAttrs):
        t2 = C.add(t2, C.mul(h, ra))
    t3 = C.add(C.mul(ipk["h_sk"], rSk), C.mul(ipk["h_rand"], rRNym))
    a_eid, a_rh = cred["attrs"][EID_INDEX], cred["attrs"][RH_INDEX]
    r_eid, r_rh = R(), R()
    EidNym = C.add(C.mul(ipk["h_attrs"][EID_INDEX], a_eid), C.mul(ipk["h_rand"], r_eid))
    RhNym = C.add(C.mul(ipk["h_attrs"][RH_INDEX], a_rh), C.mul(ipk["h_rand"], r_rh))
    rr_eid, rr_rh = R(), R()
    t4 = C.add(C.mul(ipk["h_attrs"][EID_INDEX], rAttrs[EID_INDEX]), C.mul(ipk["h_rand"], rr_eid))
    t5 = C.add(C.mul(ipk["h_attrs"][RH_INDEX], rAttrs[RH_INDEX]), C.mul(ipk["h_rand"], rr_rh))
    c, _ = _challenge(C, ipk["hash"], [t1, t2, t3, APrime, ABar, BPrime, Nym, EidNym, t4, RhNym, t5], nonce)
    sig = {
        "APrime": APrime, "ABar": ABar, "BPrime": BPrime, "Nym": Nym, "c": c, "nonce": nonce,
        "sSk": (rSk + c * sk) % r, "sE": (re - c * E) % r, "sR2": (rR2 + c * r2) % r,
        "sR3": (rR3 - c * r3) % r, "sSPrime": (rSP + c * sPrime) % r, "sRNym": (rRNym + c * rnym) % r,
        "sAttrs": [(ra + c * a) % r for ra, a in zip(rAttrs, cred["attrs"])],
        "EidNym": None if "eid" in drop else EidNym, "sEid": (rr_eid + c * r_eid) % r,
        "RhNym": None if "rh" in drop else RhNym, "sRh": (rr_rh + c * r_rh) % r,
        "rev_alg": rev_alg, "epoch": epoch, "epoch_pk": curve_pr.g2_gen,
    }
    return sig, Nym


# ------------------------------------------------------------------ verify
def _g1_proto(C, raw):
    """translator G1FromProto: ECP{x, y} with 32-byte coordinates, decoded with the
    curve's G1 rules (canonical, on the curve; BN254: zeros = identity) -- the same
    rules as the nym key (unpinned for the proof's points)"""
    if raw is None:
        raise I.PointError("nil ECP")
    f = I.pb_fields(raw)
    x, y = I._pb_bytes(f, 1), I._pb_bytes(f, 2)
    if len(x) != 32 or len(y) != 32:
        raise I.PointError("ECP coordinate length")
    return C.g1_from_bytes(x + y if C is I.BN254C else b"\x04" + x + y)


def decode_signature(raw, C):
    """-> dict of the parsed fields (raises ValueError / PointError)"""
    f = I.pb_fields(raw)
    for ff, wt, _ in f:  # wire types of the known fields (proto.Unmarshal rejects a mismatch)
        if (1 <= ff <= 19 and ff != 16 and wt != 2) or (ff == 16 and wt != 0):
            raise ValueError("wire type")

    def last(k):
        v = None
        for ff, wt, val in f:
            if ff == k:
                if wt != 2:
                    raise ValueError("wire type")
                v = val
        return v
    zr = C.zr_from_field
    d = {"APrime": last(1), "ABar": last(2), "BPrime": last(3), "Nym": last(12)}
    for k, n in (("c", 4), ("sSk", 5), ("sE", 6), ("sR2", 7), ("sR3", 8), ("sSPrime", 9), ("nonce", 11),
                 ("sRNym", 13)):
        d[k] = zr(last(n) or b"")
    d["sAttrs"] = [zr(v) for ff, _, v in f if ff == 10]
    if d["nonce"] >> 256:  # mathlib BigToBytes panics on a Zr wider than 32 bytes
        raise ValueError("nonce")
    d["epoch_pk"] = last(14)
    nr = last(17)
    d["rev_alg"] = 0
    if nr:
        for ff, wt, val in I.pb_fields(nr):
            if (ff == 1 and wt != 0) or (ff == 2 and wt != 2):
                raise ValueError("wire type")
            if ff == 1:
                d["rev_alg"] = val
    for key, fld, skey in (("EidNym", 18, "sEid"), ("RhNym", 19, "sRh")):
        sub = last(fld)
        if sub is None:
            d[key], d[skey] = None, 0
        else:
            sf = I.pb_fields(sub)
            if any(ff in (1, 2) and wt != 2 for ff, wt, _ in sf):
                raise ValueError("wire type")
            d[key] = I._pb_bytes(sf, 1)
            d[skey] = zr(I._pb_bytes(sf, 2))
    return d


def verify_proof(ipk, curve_pr, W, raw):
    """Identity.verifyProof (id.go:74-108) -> None or IdentityError"""
    C = ipk["curve"]
    if not raw:  # bccsp: "invalid signature, it must not be empty" (before Unmarshal)
        raise IdentityError(E_ID_MALFORMED)
    try:
        d = decode_signature(raw, C)
    except (ValueError, I.PointError):
        raise IdentityError(E_ID_MALFORMED)
    if d["EidNym"] is None:
        raise IdentityError(E_ID_NO_EIDNYM)
    if d["RhNym"] is None:
        raise IdentityError(E_ID_NO_RHNYM)
    try:
        APrime, ABar, BPrime, Nym = (_g1_proto(C, d[k]) for k in ("APrime", "ABar", "BPrime", "Nym"))
        EidNym, RhNym = _g1_proto(C, d["EidNym"]), _g1_proto(C, d["RhNym"])
        if len(d["sAttrs"]) != N_ATTRS:
            raise ValueError("s-values")
        if d["epoch_pk"] is None:
            raise I.PointError("nil epoch pk")
        parse_ecp2(curve_pr, d["epoch_pk"])
    except (ValueError, I.PointError):
        raise IdentityError(E_ID_MALFORMED)
    if d["rev_alg"] != 0:
        raise IdentityError(E_ID_REVOCATION)
    if APrime is None:
        raise IdentityError(E_ID_APRIME)
    if not curve_pr.pairing_product_is_one([(W, APrime), (curve_pr.g2_neg(curve_pr.g2_gen), ABar)]):
        raise IdentityError(E_ID_PAIRING)
    c, r = d["c"], C.r
    nc = (-c) % r
    HR, HS, HA = ipk["h_rand"], ipk["h_sk"], ipk["h_attrs"]
    t1 = C.add(C.add(C.mul(APrime, d["sE"]), C.mul(HR, d["sR2"])), C.mul(C.add(ABar, C.neg(BPrime)), nc))
    t2 = C.add(C.mul(HR, d["sSPrime"]), C.add(C.mul(BPrime, d["sR3"]), C.mul(HS, d["sSk"])))
    for h, s in zip(HA, d["sAttrs"]):
        t2 = C.add(t2, C.mul(h, s))
    t2 = C.add(t2, C.mul((1, 2), c))
    t3 = C.add(C.add(C.mul(HS, d["sSk"]), C.mul(HR, d["sRNym"])), C.mul(Nym, nc))
    t4 = C.add(C.add(C.mul(HA[EID_INDEX], d["sAttrs"][EID_INDEX]), C.mul(HR, d["sEid"])), C.mul(EidNym, nc))
    t5 = C.add(C.add(C.mul(HA[RH_INDEX], d["sAttrs"][RH_INDEX]), C.mul(HR, d["sRh"])), C.mul(RhNym, nc))
    c2, _ = _challenge(C, ipk["hash"], [t1, t2, t3, APrime, ABar, BPrime, Nym, EidNym, t4, RhNym, t5], d["nonce"])
    if c2 != c:
        raise IdentityError(E_ID_ZK)


def verify_identity(ipk, curve_pr, W, serialized):
    """Deserializer.Deserialize(raw, true) validity part -> None or IdentityError"""
    C = ipk["curve"]
    if not serialized:
        raise IdentityError(E_ID_MALFORMED)
    try:
        f = I.pb_fields(serialized)
        nym = I._pb_bytes(f, 1)
        proof = I._pb_bytes(f, 4)
    except ValueError:
        raise IdentityError(E_ID_MALFORMED)
    if not nym:
        raise IdentityError(E_ID_MALFORMED)
    try:
        C.g1_from_bytes(nym)
    except I.PointError:
        raise IdentityError(E_ID_BADNYM)
    verify_proof(ipk, curve_pr, W, proof)
