"""Generate tests/golden/idemix_identity_golden.json: idemix owner identities
(SerializedIdemixIdentity with the association proof) made by the oracle from the
reference's OWN credentials -- the SignerConfig fixtures copied unchanged into
tests/golden/idemix/ (charlie.ExtraId2: BN254; the zkatdlog validator's user:
FP256BN) -- each with the oracle's verdict (oracle/idemix_identity.py).

The credentials and the pairing equation are pinned by the fixtures (the
credential verifies, tests/test_idemix_identity_oracle.py); the proof transcript
layout is restated (unpinned, see the oracle's header).

    python tests/golden/make_idemix_identity_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import idemix as I, idemix_identity as ID, pairing as PR  # noqa: E402

OUT = os.path.join(HERE, "idemix_identity_golden.json")
CURVES = [("bn254", "bn254_charlie", I.BN254C, PR.BN254, 1), ("fp256bn", "fp256bn_validator", I.FP256BNC, PR.FP256BN, 0)]


def _raw(*p):
    with open(os.path.join(HERE, "idemix", *p), "rb") as f:
        return f.read()


def material(d, C, PC):
    ipk_raw = _raw(d, "IssuerPublicKey")
    ipk = I.parse_ipk(ipk_raw, C)
    cred = ID.parse_signer_config(_raw(d, "SignerConfig"), C)
    return ipk_raw, ipk, cred, ID.ipk_w(PC, ipk_raw)


def verdict(ipk, PC, W, ser):
    try:
        ID.verify_identity(ipk, PC, W, ser)
        return None
    except ID.IdentityError as e:
        return str(e)


def cases(ipk, cred, C, PC, seed):
    rng = random.Random(seed)
    out = []

    def honest(tag):
        sig, nym = ID.sign(ipk, cred, rng.randrange(1, C.r), rng, PC)
        return sig, nym

    def add(name, sig, nym, nym_bytes=None, proof=None, identity=None):
        if identity is None:
            p = ID.encode_signature(sig, PC) if proof is None else proof
            identity = ID.serialize_identity(C.g1_bytes(nym) if nym_bytes is None else nym_bytes, p)
        out.append((name, identity))

    for k in range(3):
        s, n = honest(k)
        add("honest_%d" % k, s, n)
    s, n = honest(9)
    add("tampered_sE", dict(s, sE=(s["sE"] + 1) % C.r), n)
    add("tampered_c", dict(s, c=(s["c"] + 1) % C.r), n)
    add("tampered_nonce", dict(s, nonce=(s["nonce"] + 1) % C.r), n)
    add("tampered_sAttr_eid", dict(s, sAttrs=s["sAttrs"][:2] + [(s["sAttrs"][2] + 1) % C.r] + s["sAttrs"][3:]), n)
    add("tampered_sRh", dict(s, sRh=(s["sRh"] + 1) % C.r), n)
    add("tampered_ABar", dict(s, ABar=C.add(s["ABar"], (1, 2))), n)
    add("tampered_APrime", dict(s, APrime=C.add(s["APrime"], (1, 2))), n)
    add("tampered_EidNym", dict(s, EidNym=C.add(s["EidNym"], (1, 2))), n)
    add("no_eidnym", dict(s, EidNym=None), n)
    add("no_rhnym", dict(s, RhNym=None), n)
    add("no_eidnym_no_rhnym", dict(s, EidNym=None, RhNym=None), n)
    add("revocation_alg_1", dict(s, rev_alg=1), n)
    add("three_s_attrs", dict(s, sAttrs=s["sAttrs"][:3]), n)
    add("no_epoch_pk", dict(s, epoch_pk=None), n)
    add("epoch_1", dict(s, epoch=1), n)  # not checked by Ver (no revocation)
    if C is I.BN254C:
        add("unreduced_sE", dict(s, sE=s["sE"] + C.r), n)  # NewZrFromBytes keeps the integer, Mul reduces
        add("c_plus_r", dict(s, c=s["c"] + C.r), n)        # Zr.Equals compares integers
        add("nonce_33_bytes", dict(s, nonce=s["nonce"] + (1 << 256)), n)
    # a proof point off the curve (BPrime.y + 1)
    bad = ID.encode_signature(dict(s, BPrime=(s["BPrime"][0], (s["BPrime"][1] + 1) % C.p)), PC)
    add("bprime_off_curve", s, n, proof=bad)
    # APrime = identity: BN254 encodes it as zeros; FP256BN (0, 0) is not a point
    if C is I.BN254C:
        ap0 = ID.encode_signature(dict(s, APrime=(0, 0)), PC)
        add("aprime_identity", s, n, proof=ap0)
    # the proof's nym need not be the identity's nym key (the restated Ver never reads it)
    s2, n2 = honest(10)
    add("other_nym_key", s, n, nym_bytes=C.g1_bytes(n2))
    # identity-level errors
    add("empty_identity", s, n, identity=b"")
    add("empty_nym", s, n, identity=I.pb_bytes_field(4, ID.encode_signature(s, PC)))
    add("nym_wrong_length", s, n, nym_bytes=C.g1_bytes(n)[:-1])
    nb = bytearray(C.g1_bytes(n))
    nb[-1] ^= 1
    add("nym_off_curve", s, n, nym_bytes=bytes(nb))
    add("empty_proof", s, n, proof=b"")
    add("garbage_proof", s, n, proof=b"\x0a\xff\xff")
    add("truncated_proof", s, n, proof=ID.encode_signature(s, PC)[:-7])
    add("extra_ou_field", s, n, identity=ID.serialize_identity(C.g1_bytes(n), ID.encode_signature(s, PC)) +
        I.pb_bytes_field(2, b"org1"))
    return out


def main():
    doc = {}
    for tag, d, C, PC, cid in CURVES:
        ipk_raw, ipk, cred, W = material(d, C, PC)
        cs = []
        for name, ident in cases(ipk, cred, C, PC, seed=hash(tag) & 0xFFFF if False else (11 if cid else 12)):
            cs.append({"name": name, "identity": ident.hex(), "error": verdict(ipk, PC, W, ident)})
            print(tag, name, cs[-1]["error"], flush=True)
        # a tile of honest identities and 1-in-8 tampered ones for the large-batch tests
        rng = random.Random(99 + cid)
        tile = []
        for k in range(64):
            sig, nym = ID.sign(ipk, cred, rng.randrange(1, C.r), rng, PC)
            if k % 8 == 5:
                sig = dict(sig, sSPrime=(sig["sSPrime"] + 1) % C.r)
            ident = ID.serialize_identity(C.g1_bytes(nym), ID.encode_signature(sig, PC))
            tile.append({"identity": ident.hex(), "error": verdict(ipk, PC, W, ident)})
        doc[tag] = {"issuer": d, "curve_id": cid, "cases": cs, "tile": tile}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
