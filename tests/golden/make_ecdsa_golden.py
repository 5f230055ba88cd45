"""Generate tests/golden/ecdsa_golden.json with the OpenSSL CLI (an independent
P-256/SHA-256 implementation) — run once in the build container:

    python3 tests/golden/make_ecdsa_golden.py

Each case: msg (hex), sig (hex DER), pkix (hex SubjectPublicKeyInfo, as in
ecdsa.Verifier.Serialize -> x509.MarshalPKIXPublicKey), pk64 (hex X||Y),
expect (status the reference's Verifier.Verify maps to,
validator/ecdsa/ecdsa.go:82-113), src ("openssl" = validity decided by
`openssl dgst -verify`; "rule" = decided by the Go encoding/asn1 / IsLowS /
ecdsa.Verify rules on top of an OpenSSL-valid signature).
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
OK, MAL, HIGHS, INV = 0, 13, 14, 15


def run(*a, inp=None):
    return subprocess.run(a, input=inp, capture_output=True, check=False)


def der_int(v):
    b = v.to_bytes((v.bit_length() + 8) // 8 or 1, "big", signed=True) if v >= 0 else \
        v.to_bytes((v.bit_length() + 8) // 8, "big", signed=True)
    return b"\x02" + bytes([len(b)]) + b


def der_sig(r, s):
    body = der_int(r) + der_int(s)
    return b"\x30" + bytes([len(body)]) + body


def parse_rs(sig):
    # openssl output is always minimal DER with short lengths
    rl = sig[3]
    r = int.from_bytes(sig[4:4 + rl], "big")
    s = int.from_bytes(sig[6 + rl:6 + rl + sig[5 + rl]], "big")
    return r, s


def main():
    cases = []
    with tempfile.TemporaryDirectory() as d:
        def ossl_verify(pub, msg, sig):
            open(os.path.join(d, "m"), "wb").write(msg)
            open(os.path.join(d, "s"), "wb").write(sig)
            r = run("openssl", "dgst", "-sha256", "-verify", pub, "-keyform", "DER", "-signature",
                    os.path.join(d, "s"), os.path.join(d, "m"))
            return r.returncode == 0
        for kid in range(4):
            kp, pub = os.path.join(d, "k%d.pem" % kid), os.path.join(d, "p%d.der" % kid)
            run("openssl", "ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", kp)
            run("openssl", "ec", "-in", kp, "-pubout", "-outform", "DER", "-out", pub)
            pkix = open(pub, "rb").read()
            assert len(pkix) == 91 and pkix[26] == 4
            for mid in range(6):
                msg = os.urandom([0, 5, 55, 64, 119, 1000][mid])
                open(os.path.join(d, "m"), "wb").write(msg)
                sig = run("openssl", "dgst", "-sha256", "-sign", kp, os.path.join(d, "m")).stdout
                assert ossl_verify(pub, msg, sig)
                r, s = parse_rs(sig)
                lo, hi = (s, N - s) if s <= N // 2 else (N - s, s)
                sig_lo, sig_hi = der_sig(r, lo), der_sig(r, hi)
                assert ossl_verify(pub, msg, sig_lo) and ossl_verify(pub, msg, sig_hi)

                def add(m, sg, exp, src, pk=pkix, tag=""):
                    cases.append({"msg": m.hex(), "sig": sg.hex(), "pkix": pk.hex(), "pk64": pk[27:].hex(),
                                  "expect": exp, "src": src, "tag": tag})
                add(msg, sig_lo, OK, "openssl", tag="valid low-S")
                add(msg, sig_hi, HIGHS, "rule", tag="valid high-S")
                bad = msg + b"x"
                assert not ossl_verify(pub, bad, sig_lo)
                add(bad, sig_lo, INV, "openssl", tag="tampered message")
                sig_r = der_sig(r ^ 1, lo)
                assert not ossl_verify(pub, msg, sig_r)
                add(msg, sig_r, INV, "openssl", tag="tampered r")
                if mid == 0:
                    add(msg, sig_lo + b"\x00\x01", OK, "rule", tag="trailing bytes after SEQUENCE (ignored by asn1.Unmarshal)")
                    body = sig_lo[2:] + b"\x05\x00"
                    add(msg, b"\x30" + bytes([len(body)]) + body, OK, "rule", tag="extra element in SEQUENCE")
                    add(msg, sig_lo[:-1], MAL, "rule", tag="truncated")
                    add(msg, b"\x30\x81" + bytes([len(sig_lo) - 2]) + sig_lo[2:], MAL, "rule", tag="non-minimal length")
                    add(msg, b"\x30\x80" + sig_lo[2:] + b"\x00\x00", MAL, "rule", tag="indefinite length")
                    rb = r.to_bytes(32, "big")
                    body = b"\x02\x21\x00" + rb + der_int(lo)
                    exp = MAL if rb[0] < 0x80 else OK
                    add(msg, b"\x30" + bytes([len(body)]) + body, exp, "rule", tag="r with leading zero")
                    add(msg, b"", MAL, "rule", tag="empty")
                    add(msg, der_sig(r, -lo), INV, "rule", tag="negative s")
                    add(msg, der_sig(-r, lo), INV, "rule", tag="negative r")
                    add(msg, der_sig(r, 0), INV, "rule", tag="s = 0")
                    add(msg, der_sig(0, lo), INV, "rule", tag="r = 0")
                    add(msg, der_sig(r + N, lo), INV, "rule", tag="r + n")
                    add(msg, der_sig(r, lo + N), HIGHS, "rule", tag="s + n")
                    offc = bytearray(pkix)
                    offc[-1] ^= 1
                    add(msg, sig_lo, INV, "rule", pk=bytes(offc), tag="off-curve public key")
    json.dump({"curve": "P-256", "generator": "OpenSSL " + run("openssl", "version").stdout.decode().strip(),
               "cases": cases}, open(os.path.join(HERE, "ecdsa_golden.json"), "w"), indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    sys.exit(main())
