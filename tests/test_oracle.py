"""CPU: the oracle pinned against the reference's own fixture (KAT-1) and
against the committed golden vectors."""
import json
import os

import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, der, zkat


def test_kat1_public_params_fields(oracle_pp):
    """cmd/tokengen/testdata/zkatdlog_pp.json decodes as setup.go:319-372 says."""
    pp = oracle_pp
    assert pp.label == "zkatdlog" and pp.version == "1.0.0" and pp.curve == 1
    assert len(pp.ped) == 3 and len(pp.left) == 64 and len(pp.right) == 64
    assert pp.bit_length == 64 and pp.rounds == 6 and pp.precision == 64
    assert pp.max_token == (1 << 64) - 1
    for p in pp.ped + pp.left + pp.right + [pp.P, pp.Q]:
        assert bn.on_curve(p) and p is not None


def test_kat1_hash_to_g1_generators(oracle_pp):
    """All 130 range-proof generators = HashToG1(label) (setup.go:388-406):
    RFC 9380 SVDW, expand_message_xmd(SHA-256), empty DST."""
    pp = oracle_pp
    assert bn.hash_to_g1(b"0") == pp.P
    assert bn.hash_to_g1(b"1") == pp.Q
    for i in range(64):
        assert bn.hash_to_g1(("RangeProof.%d" % (2 * (i + 1))).encode()) == pp.left[i]
        assert bn.hash_to_g1(("RangeProof.%d" % (2 * (i + 1) + 1)).encode()) == pp.right[i]


def test_kat1_spot_values(oracle_pp):
    """SURVEY §8c spot prefixes of the fixture's X coordinates."""
    pp = oracle_pp
    pref = lambda p: bn.g1_bytes(p).hex()[:16]  # noqa: E731
    assert pref(pp.P) == "02ac6640d3fbbd18"
    assert pref(pp.Q) == "12b2e282fcb7ef99"
    assert pref(pp.left[0]) == "10a3446b9b5c7d3a"
    assert pref(pp.right[0]) == "0f407d97549170aa"
    assert pref(pp.ped[0]) == "00671a6b467b3245"
    assert pref(pp.ped[1]) == "0533dc6b3c728ccb"
    assert pref(pp.ped[2]) == "21c0c8b2339f1b6b"


def test_group_law_basics():
    g = bn.GEN
    assert bn.g1_mul(g, bn.R) is None
    assert bn.g1_add(bn.g1_mul(g, 5), bn.g1_mul(g, 7)) == bn.g1_mul(g, 12)
    assert bn.g1_add(g, bn.g1_neg(g)) is None
    assert bn.g1_from_bytes(bytes(64)) is None
    with pytest.raises(bn.PointError):
        bn.g1_from_bytes(bytes(63) + b"\x01")


def test_der_shapes():
    """asn1.go:27-112 encodings."""
    v = der.values([b"ab", b""])
    assert v == bytes.fromhex("3008") + bytes.fromhex("3006") + b"\x04\x02ab" + b"\x04\x00"
    assert der.unmarshal_values(v) == [b"ab", b""]
    e = der.element(1, b"\x00" * 32)
    assert der.unmarshal_element(e) == (1, b"\x00" * 32)
    with pytest.raises(der.DerError):
        der.unmarshal_element(e + b"\x00")  # trailing bytes (asn1.go:172)
    # x0 transcript framing (ipa.go:209): SEQUENCE OF OCTET STRING
    assert der.marshal_std_bytes_list([b"x", b"||"])[:2] == b"\x30\x07"


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _load("rp_golden.json"), ids=lambda c: "n%d-%s" % (c["bits"], c["tamper"] or c["value"]))
def test_oracle_rp_golden(case, oracle_pp):
    pp = oracle_pp.with_bit_length(case["bits"])
    raw = bytes.fromhex(case["proof"])
    p = zkat.RangeProof.deserialize(raw)
    assert p.serialize() == raw
    tr = {}
    V = bn.g1_from_bytes(bytes.fromhex(case["commitment"]))
    err = zkat.rp_verify(V, pp.ped[1:], pp.left, pp.right, pp.P, pp.Q, pp.rounds, pp.bit_length, p, tr)
    assert err == case["expect"]
    assert str(tr["x"]) == case["x"] and str(tr["y"]) == case["y"] and str(tr["z"]) == case["z"]
    if "com" in case:
        assert bn.g1_bytes(tr["com"]).hex() == case["com"]
        assert str(tr["x0"]) == case["x0"]


@pytest.mark.parametrize("case", _load("transfer_golden.json"), ids=lambda c: c["name"])
def test_oracle_transfer_golden(case, oracle_pp):
    pp = oracle_pp.with_bit_length(case["bits"])
    ins = [bn.g1_from_bytes(bytes.fromhex(h)) for h in case["inputs"]]
    outs = [bn.g1_from_bytes(bytes.fromhex(h)) for h in case["outputs"]]
    err, idx = zkat.transfer_verify(pp, ins, outs, bytes.fromhex(case["proof"]))
    assert (err, idx) == (case["expect"], case["index"])


@pytest.mark.parametrize("case", _load("issue_golden.json"), ids=lambda c: c["name"])
def test_oracle_issue_golden(case, oracle_pp):
    pp = oracle_pp.with_bit_length(case["bits"])
    toks = [bn.g1_from_bytes(bytes.fromhex(h)) for h in case["tokens"]]
    err, idx = zkat.issue_verify(pp, toks, bytes.fromhex(case["proof"]))
    assert (err, idx) == (case["expect"], case["index"])


def test_c_oracle_msm_matches_python_oracle():
    """The C MSM baseline (bench.py --workload msm cpu_baseline) equals the
    Python restatement of sum (k mod r) P (G1.Mul + Add), incl. identities."""
    import random

    from oracle import bn254 as bn, cref

    rng = random.Random(0xC3C)
    pts = [bn.g1_mul(bn.GEN, rng.randrange(1, bn.R)) for _ in range(12)] + [None]
    sc = [rng.getrandbits(256) for _ in range(12)] + [5]
    blob = b"".join(bn.g1_bytes(p) for p in pts)
    sblob = b"".join(k.to_bytes(32, "big") for k in sc)
    assert cref.msm(blob, sblob, threads=3) == bn.g1_bytes(bn.g1_msm(pts, sc))
    P = pts[0]
    assert cref.msm(bn.g1_bytes(P) * 2, (7).to_bytes(32, "big") + (bn.R - 7).to_bytes(32, "big")) == bytes(64)
