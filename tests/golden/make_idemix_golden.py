"""Generate tests/golden/idemix_golden.json: idemix nym signatures over the
BN254 issuer key of cmd/tokengen/testdata/idemix (the key the benchmark's
public parameters, zkatdlog_pp.json, carry) and over the FP256BN_AMCL key of
nogh/v1/validator/testdata/idemix (the validator tests' key), made and decided by the oracle
(oracle/idemix.py, seeded).  Honest signatures plus the tamperings a verifier
must reject, with the reference's error strings.

    python tests/golden/make_idemix_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bn254, idemix  # noqa: E402


def make(raw, curve, seed):
    ipk = idemix.parse_ipk(raw, curve)
    C = curve
    rng = random.Random(seed)
    cases = []

    def add(name, nym, sig, msg):
        try:
            idemix.nym_verify(ipk, nym, sig, msg)
            err = None
        except idemix.NymError as e:
            err = str(e)
        cases.append({"name": name, "nym": nym.hex(), "sig": sig.hex(), "msg": msg.hex(), "error": err})

    for i, ml in enumerate([0, 1, 27, 28, 55, 56, 63, 64, 91, 92, 119, 120, 200, 1000, 4099]):
        sk, rn = rng.randrange(C.r), rng.randrange(C.r)
        nym = idemix.make_nym(ipk, sk, rn)
        msg = bytes(rng.randrange(256) for _ in range(ml))
        sig = idemix.nym_sign(ipk, sk, nym, rn, msg, rng)
        nb = C.g1_bytes(nym)
        add("honest_len%d" % ml, nb, sig, msg)
        if i % 3 == 0:
            add("msg_flip_len%d" % ml, nb, sig, (msg[:-1] + bytes([msg[-1] ^ 1])) if msg else b"\0")
        if i % 3 == 1:
            c, s1, s2, nonce = idemix.decode_nym_sig(sig, C)
            add("s_sk_plus1_len%d" % ml, nb, idemix.encode_nym_sig(c, (s1 + 1) % C.r, s2, nonce), msg)
            add("nonce_plus1_len%d" % ml, nb, idemix.encode_nym_sig(c, s1, s2, nonce + 1), msg)
            if s1 + C.r < 1 << 256:
                add("s_sk_unreduced_len%d" % ml, nb, idemix.encode_nym_sig(c, s1 + C.r, s2, nonce), msg)
            if c + C.r < 1 << 256:
                add("c_unreduced_len%d" % ml, nb, idemix.encode_nym_sig(c + C.r, s1, s2, nonce), msg)
        if i % 3 == 2:
            other = C.g1_bytes(idemix.make_nym(ipk, sk + 1, rn))
            add("wrong_nym_len%d" % ml, other, sig, msg)
            add("truncated_sig_len%d" % ml, nb, sig[:-5], msg)
            add("empty_sig_len%d" % ml, nb, b"", msg)
            off = bytearray(nb)
            off[-1] ^= 1
            add("nym_off_curve_len%d" % ml, bytes(off), sig, msg)
            add("nym_short_len%d" % ml, nb[:-1], sig, msg)
            c, s1, s2, nonce = idemix.decode_nym_sig(sig, C)
            if C is idemix.BN254C:
                add("nonce_too_wide_len%d" % ml, nb, idemix.encode_nym_sig(c, s1, s2, nonce + (1 << 256)), msg)
            else:  # AMCL FromBytes reads the first 32 bytes of a field; a shorter one panics
                f = idemix.pb_fields(sig)
                short = b"".join(idemix.pb_bytes_field(k, v[1:] if k == 3 else v) for k, _, v in f)
                add("short_field_len%d" % ml, nb, short, msg)
                longer = b"".join(idemix.pb_bytes_field(k, v + b"\x07" if k == 2 else v) for k, _, v in f)
                add("long_field_len%d" % ml, nb, longer, msg)
    return {"curve": C.name, "ipk": raw.hex(), "cases": cases}


def main():
    out = {"source": "oracle/idemix.py via tests/golden/make_idemix_golden.py (seeds 0x1DE41, 0x1DE42)"}
    raw = open(os.path.join(HERE, "idemix", "bn254_tokengen", "IssuerPublicKey"), "rb").read()
    out["bn254"] = make(raw, idemix.BN254C, 0x1DE41)
    raw = open(os.path.join(HERE, "idemix", "fp256bn_validator", "IssuerPublicKey"), "rb").read()
    out["fp256bn"] = make(raw, idemix.FP256BNC, 0x1DE42)
    with open(os.path.join(HERE, "idemix_golden.json"), "w") as f:
        json.dump(out, f, indent=0)
    for k in ("bn254", "fp256bn"):
        cs = out[k]["cases"]
        print(k, len(cs), "cases;", sum(c["error"] is None for c in cs), "accept")


if __name__ == "__main__":
    main()
