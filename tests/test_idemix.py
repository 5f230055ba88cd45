"""Idemix owner signatures (the idemix half):
crypto.NymSignatureVerifier.Verify (services/identity/idemix/crypto/id.go:145-161).

CPU tests cover the library's host parsing (SerializedIdemixIdentity) and that
the issuer key in the benchmark's public parameters is the BN254 tokengen key
the fixtures use.  GPU tests run fts_nym_verify_batch through the C-ABI and
compare every verdict with tests/golden/idemix_golden.json and with the oracle
(oracle/idemix.py) on seeded random batches."""
import base64
import json
import os
import random

import pytest

from conftest import GOLDEN, PP_PATH

with open(os.path.join(GOLDEN, "idemix_golden.json")) as f:
    GOLD_ALL = json.load(f)
GOLD = GOLD_ALL["bn254"]
IPK = bytes.fromhex(GOLD["ipk"])
GOLD_FBN = GOLD_ALL["fp256bn"]
IPK_FBN = bytes.fromhex(GOLD_FBN["ipk"])


def test_pp_carries_the_fixture_issuer_key():
    # zkatdlog_pp.json (cmd/tokengen/testdata) holds this BN254 idemix issuer key (curve id 1)
    with open(PP_PATH) as f:
        raw = base64.b64decode(json.load(f)["raw"])
    i = raw.find(IPK)
    assert i > 0
    assert raw[i + len(IPK):i + len(IPK) + 4] == bytes([0x12, 0x02, 0x08, 0x01])


def test_identity_nym_parse():
    from fts_gpu import idemix as I
    from oracle import idemix as O
    nym = bytes(range(64))
    ser = O.serialize_identity(nym, ou=b"org1", role=b"\x08\x01", proof=b"p" * 300)
    assert I.identity_nym(ser) == nym == O.identity_nym(ser)
    with pytest.raises(Exception):
        I.identity_nym(O.serialize_identity(b"", ou=b"org1"))
    with pytest.raises(Exception):
        I.identity_nym(ser[:-5])


@pytest.fixture(scope="module")
def ipk_dev():
    from fts_gpu import idemix as I
    k = I.IssuerKey(IPK, device=0)
    yield k
    k.close()


@pytest.fixture(scope="module")
def ipk_fbn():
    from fts_gpu import idemix as I
    k = I.IssuerKey(IPK_FBN, device=0, curve=I.FTS_CURVE_FP256BN_AMCL)
    yield k
    k.close()


def _golden(dev, gold):
    from fts_gpu import idemix as I
    cases = gold["cases"]
    st = dev.verify_batch([bytes.fromhex(c["nym"]) for c in cases], [bytes.fromhex(c["sig"]) for c in cases],
                          [bytes.fromhex(c["msg"]) for c in cases])
    for c, s in zip(cases, st):
        assert I.message(int(s)) == c["error"], c["name"]
    assert sum(c["error"] is None for c in cases) == int((st == 0).sum())


@pytest.mark.gpu
def test_golden_verdicts(ipk_dev):
    _golden(ipk_dev, GOLD)


@pytest.mark.gpu
def test_golden_verdicts_fp256bn(ipk_fbn):
    _golden(ipk_fbn, GOLD_FBN)


@pytest.mark.gpu
def test_random_batch_fp256bn_against_oracle(ipk_fbn):
    from fts_gpu import idemix as I
    nyms, sigs, msgs, want = _batch(200, seed=21, curve="fp256bn")
    st = ipk_fbn.verify_batch(nyms, sigs, msgs)
    assert [I.message(int(s)) for s in st] == want


@pytest.mark.gpu
def test_single_verifier_api(ipk_dev):
    from fts_gpu import idemix as I
    c = next(c for c in GOLD["cases"] if c["error"] is None)
    v = I.NymSignatureVerifier(ipk_dev, bytes.fromhex(c["nym"]))
    v.Verify(bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"]))
    with pytest.raises(I.SignatureError, match="zero-knowledge proof is invalid"):
        v.Verify(bytes.fromhex(c["msg"]) + b"!", bytes.fromhex(c["sig"]))
    with pytest.raises(I.SignatureError, match="error unmarshalling signature"):
        v.Verify(b"m", b"")


def _batch(n, seed, nkeys=6, tamper=0.1, curve="bn254"):
    from oracle import idemix as O
    C = O.BN254C if curve == "bn254" else O.FP256BNC
    ipk = O.parse_ipk(IPK if curve == "bn254" else IPK_FBN, C)
    rng = random.Random(seed)
    keys = []
    for _ in range(nkeys):
        sk, rn = rng.randrange(C.r), rng.randrange(C.r)
        keys.append((sk, rn, O.make_nym(ipk, sk, rn)))
    nyms, sigs, msgs, want = [], [], [], []
    shared = bytes(rng.randrange(256) for _ in range(700))  # one request message, many inputs
    for i in range(n):
        sk, rn, nym = keys[rng.randrange(nkeys)]
        msg = shared if i % 2 else bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300)))
        sig = O.nym_sign(ipk, sk, nym, rn, msg, rng)
        nb = C.g1_bytes(nym)
        if rng.random() < tamper:
            kind = rng.randrange(3)
            if kind == 0:
                msg = msg + b"x"
            elif kind == 1:
                c, s1, s2, nonce = O.decode_nym_sig(sig, C)
                sig = O.encode_nym_sig(c, s1, (s2 + 1) % C.r, nonce)
            else:
                nb = C.g1_bytes(keys[(keys.index((sk, rn, nym)) + 1) % nkeys][2])
        try:
            O.nym_verify(ipk, nb, sig, msg)
            w = None
        except O.NymError as e:
            w = str(e)
        nyms.append(nb)
        sigs.append(sig)
        msgs.append(msg)
        want.append(w)
    return nyms, sigs, msgs, want


@pytest.mark.gpu
def test_random_batch_against_oracle(ipk_dev):
    from fts_gpu import idemix as I
    nyms, sigs, msgs, want = _batch(300, seed=11)
    st = ipk_dev.verify_batch(nyms, sigs, msgs)
    assert [I.message(int(s)) for s in st] == want
    assert 0 < sum(w is not None for w in want) < 300


@pytest.mark.gpu
def test_large_batch_packed_tiled(ipk_dev):
    """65,536 signatures (a tiled 256-signature oracle batch): verdicts exact at every position."""
    _tiled(ipk_dev, "bn254")


@pytest.mark.gpu
def test_large_batch_packed_tiled_fp256bn(ipk_fbn):
    """The FP256BN kernel (GLV chain, per-lane tables strided over 65,536 lanes) at full size."""
    _tiled(ipk_fbn, "fp256bn")


def _tiled(dev, curve):
    import numpy as np
    nyms, sigs, msgs, want = _batch(256, seed=12, tamper=0.05, curve=curve)
    reps = 256
    n = 256 * reps
    nym_buf = b"".join(nyms) * reps
    sig_buf, msg_buf = b"".join(sigs), b"".join(msgs)
    so = np.cumsum([0] + [len(s) for s in sigs[:-1]]).astype(np.uint64)
    mo = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint64)
    sl = np.array([len(s) for s in sigs], dtype=np.uint64)
    ml = np.array([len(m) for m in msgs], dtype=np.uint64)
    st = dev.verify_packed(nym_buf, sig_buf, np.tile(so, reps), np.tile(sl, reps), msg_buf, np.tile(mo, reps),
                           np.tile(ml, reps))
    exp = np.tile(np.array([w is None for w in want]), reps)
    assert st.shape == (n,)
    assert ((st == 0) == exp).all()


@pytest.mark.gpu
def test_packed_bounds_checked(ipk_dev):
    import numpy as np
    with pytest.raises(ValueError):
        ipk_dev.verify_packed(b"\0" * 64, b"abc", np.array([0]), np.array([10]), b"", np.array([0]), np.array([0]))
    with pytest.raises(ValueError):
        ipk_dev.verify_packed(b"\0" * 10, b"abc", np.array([0]), np.array([3]), b"", np.array([0]), np.array([0]))


@pytest.mark.gpu
def test_bad_issuer_key_rejected():
    from fts_gpu import idemix as I
    from fts_gpu import _lib as L
    with pytest.raises(L.FtsError):
        I.IssuerKey(IPK[:100], device=0)
    with pytest.raises(L.FtsError):  # a BN254 key read as FP256BN: HSk is not on that curve
        I.IssuerKey(IPK, device=0, curve=I.FTS_CURVE_FP256BN_AMCL)
    with pytest.raises(L.FtsError):
        I.IssuerKey(IPK_FBN, device=0, curve=I.FTS_CURVE_BN254)


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["bn254", "fp256bn"])
def test_launch_tiling_gives_same_verdicts(curve):
    """the GLV lane tables are sized for one launch tile, not for n; a
    call above the tile runs several launches on the slot's stream.  A key built
    with FTS_NYM_TILE=64 (ragged last tile: 300 = 4 x 64 + 44) must return the
    oracle's verdicts at every position."""
    import os

    from fts_gpu import idemix as I
    old = os.environ.get("FTS_NYM_TILE")
    os.environ["FTS_NYM_TILE"] = "64"
    try:
        k = I.IssuerKey(IPK if curve == "bn254" else IPK_FBN, device=0,
                        curve=I.FTS_CURVE_BN254 if curve == "bn254" else I.FTS_CURVE_FP256BN_AMCL)
    finally:
        if old is None:
            del os.environ["FTS_NYM_TILE"]
        else:
            os.environ["FTS_NYM_TILE"] = old
    nyms, sigs, msgs, want = _batch(300, seed=31, curve=curve)
    st = k.verify_batch(nyms, sigs, msgs)
    k.close()
    assert [I.message(int(s)) for s in st] == want
    assert 0 < sum(w is not None for w in want) < 300


class _ZeroNonces:
    """rng for nym_sign whose commitment nonces are 0 (t = O), nonce field random"""
    def __init__(self, seed):
        self.r, self.calls = random.Random(seed), 0

    def randrange(self, n):
        self.calls += 1
        return self.r.randrange(n) if self.calls == 1 else 0


def test_zero_nonce_signature_oracle():
    """a signer with zero commitment nonces gets t = O; the transcript then
    carries the curve's encoding of infinity (FP256BN: AMCL ToBytes of its
    projective (0, 1, 0) = 0x04 || 0 || 1) and the signature is valid"""
    from oracle import idemix as O
    for C, ipk_raw in ((O.FP256BNC, IPK_FBN), (O.BN254C, IPK)):
        ipk = O.parse_ipk(ipk_raw, C)
        sk, rn = 12345, 67890
        nym = O.make_nym(ipk, sk, rn)
        sig = O.nym_sign(ipk, sk, nym, rn, b"zero nonces", _ZeroNonces(3))
        O.nym_verify(ipk, C.g1_bytes(nym), sig, b"zero nonces")
    assert O.FP256BNC.g1_bytes(None) == b"\x04" + bytes(32) + (1).to_bytes(32, "big")


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["bn254", "fp256bn"])
def test_zero_nonce_signature_gpu(curve, ipk_dev, ipk_fbn):
    """t = O on the device: the same verdicts as the oracle (valid, and invalid
    for a different message)"""
    from fts_gpu import idemix as I
    from oracle import idemix as O
    C, raw, dev = (O.BN254C, IPK, ipk_dev) if curve == "bn254" else (O.FP256BNC, IPK_FBN, ipk_fbn)
    ipk = O.parse_ipk(raw, C)
    sk, rn = 424242, 171717
    nym = O.make_nym(ipk, sk, rn)
    sig = O.nym_sign(ipk, sk, nym, rn, b"zero nonces", _ZeroNonces(5))
    nb = C.g1_bytes(nym)
    st = dev.verify_batch([nb, nb], [sig, sig], [b"zero nonces", b"other"])
    assert I.message(int(st[0])) is None
    assert I.message(int(st[1])) is not None
