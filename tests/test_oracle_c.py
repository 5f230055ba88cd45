"""CPU: the C restatement (oracle/c/ref_verify.c, bench.py's cpu_baseline)
pinned against the committed golden vectors of the Python oracle.

rp_golden.json: every standalone range proof (8..64 bits, honest, out of
range, tampered T1 / L0 / Left / ip) -> the same verdict class as the
reference error string recorded in the fixture (bulletproof.go:252-333,
ipa.go:190-262).
headline_golden.json: the range proofs inside the 64-bit 2-in/2-out
transfers, verified one by one against V_j = Out_j - CT as the range
goroutine of transfer.go:171-187 does, give the recorded first failing
index and class (rangecorrectness.go:141-160)."""
import json
import os

import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, cref, der, zkat

# verify_one's return codes = fts_status numbering of the library
RP_CODE = {None: 0, "invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
           "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def built():
    cref.build()


def test_c_oracle_rp_golden(built, oracle_pp):
    cases = _load("rp_golden.json")
    for bits in sorted({c["bits"] for c in cases}):
        pp = oracle_pp.with_bit_length(bits)
        sel = [c for c in cases if c["bits"] == bits]
        got = cref.rp_verify_many(pp, [bytes.fromhex(c["commitment"]) for c in sel],
                                  [bytes.fromhex(c["proof"]) for c in sel], threads=4)
        assert got == [RP_CODE[c["expect"]] for c in sel], bits


def test_c_oracle_headline_transfer_range_proofs(built, oracle_pp):
    """the C oracle on the 64-bit range proofs of the headline transfers"""
    cases = _load("headline_golden.json")["transfers"]
    for c in cases:
        raw = bytes.fromhex(c["proof"])
        tas_raw, rc_raw = der.unmarshal_values(raw)
        tas = zkat.TypeAndSumProof.deserialize(tas_raw)
        rps = der.unmarshal_values(der.unmarshal_values(rc_raw)[0])
        outs = [bn.g1_from_bytes(bytes.fromhex(h)) for h in c["outputs"]]
        coms = [bn.g1_bytes(bn.g1_sub(o, tas.CT)) for o in outs]
        got = cref.rp_verify_many(oracle_pp, coms, rps, threads=2)
        first = next(((j, s) for j, s in enumerate(got) if s != 0), None)
        if c["expect"] is None:
            assert first is None, c["name"]
        elif c["expect"].startswith("invalid range proof at index"):
            inner = c["expect"].split(": ", 1)[1]
            assert first == (c["index"], RP_CODE[inner]), c["name"]
        else:  # TypeAndSum failures: the range proofs themselves are honest
            assert first is None, c["name"]


def test_c_oracle_headline_actions(built, oracle_pp):
    """the C oracle's whole transfer / issue verifier (bench cpu_baseline of C4/C5)
    on the headline fixtures: same verdict class and fail index as the Python oracle"""
    head = _load("headline_golden.json")
    from fts_gpu_msgs import classify
    tr = [("transfer", [bytes.fromhex(h) for h in c["inputs"]], [bytes.fromhex(h) for h in c["outputs"]],
           bytes.fromhex(c["proof"])) for c in head["transfers"]]
    got = cref.action_verify_many(oracle_pp, tr, threads=4)
    assert got == [classify(c["expect"], c["index"]) for c in head["transfers"]]
    p32 = oracle_pp.with_bit_length(32)
    iss = [("issue", [], [bytes.fromhex(h) for h in c["tokens"]], bytes.fromhex(c["proof"])) for c in head["issues"]]
    got = cref.action_verify_many(p32, iss, threads=4)
    assert got == [classify(c["expect"], c["index"]) for c in head["issues"]]


def test_cpu_batch_rp_golden(built, oracle_pp):
    """the optimized CPU batch baseline (oracle/c/cpu_batch.c, bench.py's
    "optimized_batch" column): honest batches close the random linear
    combination without any per-proof fallback (so its exact com / x0 / GLV
    chain match the reference's transcript), and batches with tampered proofs
    bisect to the reference-order verdicts"""
    cases = _load("rp_golden.json")
    for bits in sorted({c["bits"] for c in cases}):
        pp = oracle_pp.with_bit_length(bits)
        cb = cref.CpuBatch(pp, window_bits=8, threads=4)
        sel = [c for c in cases if c["bits"] == bits]
        honest = [c for c in sel if c["expect"] is None]
        got, nfb = cb.verify([bytes.fromhex(c["commitment"]) for c in honest],
                             [bytes.fromhex(c["proof"]) for c in honest], threads=4)
        assert got == [0] * len(honest) and nfb == 0, bits
        # honest proofs around the tampered ones, several times over (bisection)
        mix = honest * 3 + sel + honest * 2
        got, nfb = cb.verify([bytes.fromhex(c["commitment"]) for c in mix], [bytes.fromhex(c["proof"]) for c in mix],
                             threads=3)
        assert got == [RP_CODE[c["expect"]] for c in mix], bits
        assert nfb < len(mix) or all(c["expect"] for c in sel), bits
        cb.close()


def test_cpu_pippenger_matches_term_by_term():
    """oracle/c/cpu_batch.c cpu_msm_pippenger (the C3 CPU baseline): the same group
    element as the term-by-term G1.Mul + Add oracle, with identities, scalars >= r
    and a window-count edge (n spans the c = 4 .. 11 window choices)"""
    import random

    from oracle import bn254 as bn, cref
    rng = random.Random(0xC3C3)
    for n in (1, 2, 33, 257, 3000):
        pts = [bn.g1_mul(bn.GEN, rng.randrange(1, bn.R)) for _ in range(n)]
        ks = [rng.getrandbits(256) for _ in range(n)]
        if n > 2:
            pts[1] = None          # identity
            ks[2] = bn.R           # = 0 mod r
        pb = b"".join(bn.g1_bytes(p) for p in pts)
        kb = b"".join(k.to_bytes(32, "big") for k in ks)
        assert cref.msm_pippenger(pb, kb, threads=3) == cref.msm(pb, kb, threads=3), n
    with pytest.raises(ValueError):
        cref.msm_pippenger(b"\x01" * 64, bytes(32))


def test_cpu_pippenger_widest_window():
    """2^18 points: the widest window (c = 15) with ~2^19 GLV halves x 9 windows of
    random digits, so the edge digit +2^(c-1) occurs (an int16_t digit table
    wrapped it at c = 16); P_i = (i mod 2^12 + 1) G, closed form sum k_i (i mod 2^12 + 1) G"""
    import random

    from oracle import bn254 as bn, cref
    rng = random.Random(0xC3C4)
    m, n = 1 << 12, 1 << 18
    base, P = [], None
    for i in range(m):
        P = bn.GEN if P is None else bn.g1_add(P, bn.GEN)
        base.append(bn.g1_bytes(P))
    pb = b"".join(base) * (n // m)
    ks = [rng.getrandbits(256) for _ in range(n)]
    kb = b"".join(k.to_bytes(32, "big") for k in ks)
    want = bn.g1_bytes(bn.g1_mul(bn.GEN, sum(k * (i % m + 1) for i, k in enumerate(ks)) % bn.R))
    assert cref.msm_pippenger(pb, kb, threads=8) == want
