"""FP256BN GLV constants of csrc/device/fp256bn.hpp (fbn::GlvK), used by
k_nym_verify_fbn's (r - c)*Nym chain: read from the header and checked on the
CPU against the oracle's curve (oracle/idemix.py FP256BNC): phi(x, y) =
(beta x, y) equals lambda * P, and glv_decompose's Babai rounding (restated
below limb for limb in integers) gives k = k1 + k2 lambda (mod r) with
|k1|, |k2| < 2^128 (the kernel's 33 signed 4-bit windows)."""
import os
import random
import re

from conftest import GOLDEN

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fabric-token-sdk_amd", "csrc",
                   "device", "fp256bn.hpp")
LAMBDA = 0x27311c281242030ce379baf3be321c37067081e9398533016


def _consts():
    src = open(HDR).read()
    body = src[src.index("struct GlvK"):]
    body = body[:body.index("\n};")]
    out = {}
    for name, vals in re.findall(r"(\w+)\[\d+\] = \{([^}]*)\}", body):
        limbs = [int(v.strip().rstrip("u"), 16) for v in vals.split(",")]
        out[name] = sum(l << (32 * i) for i, l in enumerate(limbs))
    return out


def _decompose(k, c, r):
    c1 = (k * c["G1"] + (1 << 383)) >> 384
    c2 = (k * c["G2"] + (1 << 383)) >> 384
    k1 = k - c1 * c["A1"] - c2 * c["A2"]
    k2 = c1 * c["NB1"] - c2 * c["A1"]
    return k1, k2


def test_fp256bn_glv_constants():
    from oracle import idemix as O
    C = O.FP256BNC
    p, r = C.p, C.r
    c = _consts()
    beta = c["BETA"] * pow(1 << 256, -1, p) % p  # out of Montgomery form
    assert pow(beta, 3, p) == 1 and beta != 1
    assert pow(LAMBDA, 3, r) == 1 and LAMBDA != 1
    # lattice: (a1, b1), (a2, b2) with b2 = a1 lie on x + y lambda = 0 (mod r)
    assert (c["A1"] - c["NB1"] * LAMBDA) % r == 0
    assert (c["A2"] + c["A1"] * LAMBDA) % r == 0
    with open(os.path.join(GOLDEN, "idemix", "fp256bn_validator", "IssuerPublicKey"), "rb") as f:
        P = O.parse_ipk(f.read(), C)["h_sk"]
    assert C.mul(P, LAMBDA) == (P[0] * beta % p, P[1])
    rng = random.Random(7)
    for k in [0, 1, 2, r - 1, r - 2, LAMBDA, r // 2] + [rng.randrange(r) for _ in range(3000)]:
        k1, k2 = _decompose(k, c, r)
        assert (k1 + k2 * LAMBDA - k) % r == 0
        assert abs(k1) < 1 << 128 and abs(k2) < 1 << 128
