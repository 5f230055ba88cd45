"""Crafted ECDSA P-256 cases for the X.x = r + n branch of Verify
(ecdsa_kernels.hip final check; Go crypto/ecdsa verifies X.x mod n == r).

Random signatures reach that branch with probability ~2^-128, so it is built
on purpose: a curve point R whose x lies in [n, p), r = x - n, any low s and
message m (e = SHA-256(m)), and the public key Q = r^-1 (s R - e G).  Then
u1 G + u2 Q = R, so (r, s) is VALID for Q.  The same signature with r
replaced by x (>= n) must be rejected by Verify's range check.
Validity is double-checked with the OpenSSL CLI (an independent
implementation).  Writes tests/golden/ecdsa_crafted_golden.json:

    python3 tests/golden/make_ecdsa_crafted.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ecdsa_p256 as O  # noqa: E402

# SubjectPublicKeyInfo prefix of an uncompressed P-256 key (x509.MarshalPKIXPublicKey)
SPKI = bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200")


def sqrt_p(a):
    y = pow(a, (O.P + 1) // 4, O.P)  # p = 3 mod 4
    return y if y * y % O.P == a % O.P else None


def main():
    cases = []
    x = O.N
    found = 0
    with tempfile.TemporaryDirectory() as d:
        while found < 3:
            y = sqrt_p(x * x * x - 3 * x + O.B)
            if y is None:
                x += 1
                continue
            R = (x, y)
            r = x - O.N
            msg = b"crafted r+n case %d" % found
            e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
            s = 0x1234567 + 7919 * found
            rinv = pow(r, -1, O.N)
            sR = O.mul(s, R)
            eG = O.mul(e % O.N, O.G)
            Q = O.mul(rinv, O._add(sR, (eG[0], (-eG[1]) % O.P)))
            pk64 = Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")
            sig = O.der_sig(r, s)
            bad = O.der_sig(x, s)
            assert O.verify(msg, sig, Q) == O.OK and O.verify(msg, bad, Q) == O.SIG_INVALID
            pub = os.path.join(d, "p.der")
            open(pub, "wb").write(SPKI + b"\x04" + pk64)
            open(os.path.join(d, "m"), "wb").write(msg)
            for sg, want in ((sig, True), (bad, False)):
                open(os.path.join(d, "s"), "wb").write(sg)
                rc = subprocess.run(["openssl", "dgst", "-sha256", "-verify", pub, "-keyform", "DER", "-signature",
                                     os.path.join(d, "s"), os.path.join(d, "m")], capture_output=True).returncode
                assert (rc == 0) == want, (found, want)
            for sg, exp, tag in ((sig, O.OK, "x(R) in [n, p): r = x - n (valid, X.x = r + n)"),
                                 (bad, O.SIG_INVALID, "x(R) in [n, p): r = x >= n (rejected by the range check)")):
                cases.append({"msg": msg.hex(), "sig": sg.hex(), "pkix": (SPKI + b"\x04" + pk64).hex(),
                              "pk64": pk64.hex(), "expect": exp, "src": "openssl", "tag": tag})
            found += 1
            x += 1
    json.dump({"curve": "P-256", "cases": cases}, open(os.path.join(HERE, "ecdsa_crafted_golden.json"), "w"),
              indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
