"""Generate tests/golden/audit_golden.json with the CPU oracle.

Token opening checks of the auditor (crypto/audit/auditor.go:226-238) and of
Token.ToClear (crypto/token/token.go:69-83): each case is an opening
(token.Data, type, value, blinding factor) and the oracle's verdict
(oracle.zkat.inspect_output).  The reference holds no opening vectors
(auditor_test.go is randomised); the commitment formula itself is the one the
transfer / issue golden proofs already pin (their tokens are commitments of
this form accepted by TypeAndSum / SameType).

    python tests/golden/make_audit_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bn254 as bn, pp as ppm, zkat  # noqa: E402

R, P = bn.R, bn.P


def be(x):
    return x.to_bytes(32, "big")


def main():
    pp = ppm.load_pp(open(os.path.join(HERE, "zkatdlog_pp.json"), "rb").read())
    ped = pp.ped
    rng = zkat.make_rng(0xF7A5_00A0)
    cases = []

    def add(name, com, ttype, value, bf):
        err = zkat.inspect_output(ped, com, ttype, value, bf)
        cases.append({"name": name, "com": com.hex() if com is not None else None, "type": ttype.hex(),
                      "value": value.hex() if value is not None else None, "bf": bf.hex() if bf is not None else None,
                      "expect": "ok" if err is None else ("malformed" if err == "malformed" else "mismatch")})

    def honest(ttype, v, bf):
        return bn.g1_bytes(zkat.token_commit(ped, ttype, v, bf))

    bf = rng.randrange(R)
    c = honest(b"ABC", 100, bf)
    add("honest", c, b"ABC", be(100), be(bf))
    bf2 = rng.randrange(R)
    add("honest_max_u64", honest(b"USD", 2**64 - 1, bf2), b"USD", be(2**64 - 1), be(bf2))
    add("wrong_value", c, b"ABC", be(101), be(bf))
    add("wrong_bf", c, b"ABC", be(100), be((bf + 1) % R))
    add("wrong_type", c, b"ABD", be(100), be(bf))
    add("unreduced_value", c, b"ABC", be(100 + R), be(bf))          # G1.Mul reduces mod r
    add("unreduced_bf", c, b"ABC", be(100), be(bf + 2 * R) if bf + 2 * R < 2**256 else be(bf + R))
    bf3 = rng.randrange(R)
    add("empty_type", honest(b"", 7, bf3), b"", be(7), be(bf3))
    long_t = bytes(rng.randrange(256) for _ in range(150))           # multi-block SHA-256
    add("long_type", honest(long_t, 12345, bf3), long_t, be(12345), be(bf3))
    add("zero_value_bf", honest(b"ABC", 0, 0), b"ABC", be(0), be(0))
    add("identity_com", bytes(64), b"ABC", be(0), be(0))
    x, y = bn.g1_from_bytes(c)
    add("negated_com", x.to_bytes(32, "big") + (P - y).to_bytes(32, "big"), b"ABC", be(100), be(bf))
    add("off_curve_com", x.to_bytes(32, "big") + ((y + 1) % P).to_bytes(32, "big"), b"ABC", be(100), be(bf))
    add("flag_bits_com", bytes([c[0] | 0x80]) + c[1:], b"ABC", be(100), be(bf))
    for k in range(1, 64):  # an honest commitment with x + p < 2^254, re-encoded with x + p
        cn = honest(b"ABC", k, bf)
        xn = int.from_bytes(cn[:32], "big")
        if xn + P < 2**254:
            add("noncanonical_x", (xn + P).to_bytes(32, "big") + cn[32:], b"ABC", be(k), be(bf))
            break
    add("nil_bf", c, b"ABC", be(100), None)
    add("nil_com", None, b"ABC", be(100), be(bf))
    for i in range(16):  # random honest / tampered mix
        v = rng.randrange(2**64)
        b = rng.randrange(R)
        t = ("T%d" % rng.randrange(4)).encode()
        com = honest(t, v, b)
        if i % 3 == 2:
            v ^= 1 << rng.randrange(64)
        add("random_%d" % i, com, t, be(v), be(b))
    with open(os.path.join(HERE, "audit_golden.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print([(c["name"], c["expect"]) for c in cases])


if __name__ == "__main__":
    main()
