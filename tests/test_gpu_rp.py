"""GPU parity: range-proof batch verification (rp/bulletproof.go:252-509,
rp/ipa.go:190-356) through the C-ABI against the oracle — verdicts AND exact
intermediates (x, y, z, polEval, x0, x_j, com, H'_i), bit-exact."""
import ctypes as C
import json
import os
import random

import pytest

from conftest import GOLDEN

from oracle import bn254 as bn, der, zkat

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "rp_golden.json")) as f:
    RP_GOLDEN = json.load(f)

STATUS_OF = {None: 0, "invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
             "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}


def _intermediates(pp, i):
    from fts_gpu import _lib as L
    k, n = pp.rounds, pp.bit_length
    ch = C.create_string_buffer(32 * (8 + 2 * k))
    com = C.create_string_buffer(64)
    hp = C.create_string_buffer(64 * n)
    L.check("dbg", L.lib.fts_debug_rp_intermediates(pp._ctx, i, ch, com, hp))
    vals = [int.from_bytes(ch.raw[32 * q:32 * q + 32], "big") for q in range(8 + 2 * k)]
    return vals, com.raw, [hp.raw[64 * q:64 * q + 64] for q in range(n)]


@pytest.mark.parametrize("bits", [8, 16, 32, 64])
def test_golden_batch_verdicts_and_intermediates(gpu_pp, bits):
    cases = [c for c in RP_GOLDEN if c["bits"] == bits]
    pp = gpu_pp(bits)
    proofs = [bytes.fromhex(c["proof"]) for c in cases]
    coms = [bytes.fromhex(c["commitment"]) for c in cases]
    st = pp.verify_range_proofs(proofs, coms)
    assert [int(s) for s in st] == [STATUS_OF[c["expect"]] for c in cases]
    for i, c in enumerate(cases):
        vals, com, hp = _intermediates(pp, i)
        assert (vals[0], vals[2], vals[4], vals[6]) == (int(c["x"]), int(c["y"]), int(c["z"]), int(c["polEval"]))
        if "com" in c:
            assert com.hex() == c["com"]
            assert [h.hex() for h in hp] == c["hprime"]
            assert vals[7] == int(c["x0"])
            assert vals[8:8 + pp.rounds] == c["xj"]


_WORK_CTX = {}


def _work_path_pp(pp_raw, bits):
    """a context whose passes all take the work path for com (FTS_COM_FIXED_MAX=0:
    Horner sum of H'_i + joint GLV/Straus chains); the default contexts run batches
    of this size on the latency path (fixed-base groups + x*D on the side stream)"""
    import fts_gpu
    if bits not in _WORK_CTX:
        old = {k: os.environ.get(k) for k in ("FTS_COM_FIXED_MAX", "FTS_LANES")}
        os.environ.update(FTS_COM_FIXED_MAX="0", FTS_LANES="1")
        try:
            _WORK_CTX[bits] = fts_gpu.PublicParams(pp_raw, bit_length=bits, device=0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return _WORK_CTX[bits]


@pytest.mark.parametrize("bits", [8, 32, 64])
def test_golden_work_path_com(pp_raw, bits):
    """the work path (large passes) computes the same com, H'_i and x0 bytes"""
    pp = _work_path_pp(pp_raw, bits)
    cases = [c for c in RP_GOLDEN if c["bits"] == bits]
    st = pp.verify_range_proofs([bytes.fromhex(c["proof"]) for c in cases],
                                [bytes.fromhex(c["commitment"]) for c in cases])
    assert [int(s) for s in st] == [STATUS_OF[c["expect"]] for c in cases]
    lt = pp.last_timings()
    assert "k_rp_com_var" in lt and "k_rp_fixed_all" not in lt
    for i, c in enumerate(cases):
        vals, com, hp = _intermediates(pp, i)
        if "com" in c:
            assert com.hex() == c["com"] and [h.hex() for h in hp] == c["hprime"] and vals[7] == int(c["x0"])


def test_latency_path_is_default_for_small_passes(gpu_pp):
    pp = gpu_pp(8)
    cases = [c for c in RP_GOLDEN if c["bits"] == 8]
    pp.verify_range_proofs([bytes.fromhex(c["proof"]) for c in cases], [bytes.fromhex(c["commitment"]) for c in cases])
    t = pp.last_timings()
    assert "k_rp_fixed_all" in t and "k_rp_xd" in t and "k_rp_com_var" not in t


def test_host_prover_batch_n64(gpu_pp, oracle_pp):
    """128 fresh proofs from the product prover, all accepted; intermediates
    of a sample match the oracle's reference-order trace."""
    pp = gpu_pp(64)
    n = 128
    vals = [(i * 0x9E3779B97F4A7C15) & ((1 << 64) - 1) for i in range(n)]
    bfs = [((i + 1) * 0x1234567).to_bytes(32, "big") for i in range(n)]
    proofs, coms = pp.prove_range_batch(vals, bfs, seed=99)
    st = pp.verify_range_proofs(proofs, coms)
    assert (st == 0).all()
    opp = oracle_pp
    for i in (0, 77):
        tr = {}
        V = bn.g1_from_bytes(coms[i])
        assert zkat.rp_verify(V, opp.ped[1:], opp.left, opp.right, opp.P, opp.Q, 6, 64,
                              zkat.RangeProof.deserialize(proofs[i]), tr) is None
        v, com, hp = _intermediates(pp, i)
        assert v[7] == tr["x0"] and com == bn.g1_bytes(tr["com"])
        assert hp == [bn.g1_bytes(h) for h in tr["Hprime"]]


def _mk(pp, value, seed):
    bf = (seed * 7919 + 1).to_bytes(32, "big")
    return pp.prove_range(value, bf, seed)


def test_tampered_and_malformed(gpu_pp, oracle_pp):
    """One batch mixing honest, tampered and malformed proofs; every verdict
    equals the reference's (oracle) error string."""
    pp = gpu_pp(8)
    opp = oracle_pp.with_bit_length(8)
    base = [_mk(pp, v, s) for v, s in ((11, 1), (22, 2), (33, 3), (44, 4), (55, 5), (66, 6))]
    proofs, coms, expect = [], [], []

    def add(raw, com):
        proofs.append(raw)
        coms.append(com)
        V = bn.g1_from_bytes(com) if com != bytes(64) else None
        try:
            rp = zkat.RangeProof.deserialize(raw)
            err = zkat.rp_verify(V, opp.ped[1:], opp.left, opp.right, opp.P, opp.Q, 3, 8, rp)
            expect.append(STATUS_OF[err])
        except zkat.Malformed:
            expect.append(1)

    raw, com = base[0]
    add(raw, com)                                                   # honest
    add(raw, base[1][1])                                            # wrong commitment
    r = zkat.RangeProof.deserialize(base[2][0]); r.data.T2 = bn.g1_neg(r.data.T2); add(r.serialize(), base[2][1])
    r = zkat.RangeProof.deserialize(base[3][0]); r.ipa.R[2] = bn.g1_add(r.ipa.R[2], opp.Q); add(r.serialize(), base[3][1])
    r = zkat.RangeProof.deserialize(base[4][0]); r.ipa.Right = (r.ipa.Right * 3) % bn.R; add(r.serialize(), base[4][1])
    r = zkat.RangeProof.deserialize(base[5][0]); r.data.Delta = (r.data.Delta + 1) % bn.R; add(r.serialize(), base[5][1])
    add(base[0][0][:-1], com)                                       # truncated DER
    add(b"", com)                                                   # empty
    # IPA with a missing round -> "invalid IPA proof" (ipa.go:195-198)
    r = zkat.RangeProof.deserialize(base[1][0]); r.ipa.L = r.ipa.L[:2]; r.ipa.R = r.ipa.R[:2]
    add(r.serialize(), base[1][1])
    # ...but the E1 failure wins when both are wrong (bulletproof.go:322 before :327)
    r = zkat.RangeProof.deserialize(base[1][0]); r.ipa.L = r.ipa.L[:2]; r.ipa.R = r.ipa.R[:2]
    add(r.serialize(), base[0][1])
    # Data with only 5 elements -> nil fields
    dvals = der.unmarshal_values(der.unmarshal_values(base[2][0])[0])
    add(der.values([der.values(dvals[:5]), der.unmarshal_values(base[2][0])[1]]), base[2][1])
    # empty IPA -> "invalid IPA proof: nil elements"
    add(der.values([der.unmarshal_values(base[3][0])[0], b""]), base[3][1])
    # point not on the curve / flag bits / non-canonical coordinate
    bad = bytearray(base[4][0]); i = bad.find(bn.g1_bytes(zkat.RangeProof.deserialize(base[4][0]).data.C))
    bad[i + 63] ^= 1; add(bytes(bad), base[4][1])
    bad = bytearray(base[4][0]); bad[i] |= 0x80; add(bytes(bad), base[4][1])
    # identity T1 (valid encoding, proof then fails E1)
    r = zkat.RangeProof.deserialize(base[5][0]); r.data.T1 = None; add(r.serialize(), base[5][1])
    # wrong curve id in an element
    good = base[0][0]
    wrong = good.replace(b"\x02\x01\x01\x04\x40", b"\x02\x01\x02\x04\x40", 1)
    add(wrong, com)
    st = pp.verify_range_proofs(proofs, coms)
    assert [int(s) for s in st] == expect


def test_empty_and_single(gpu_pp):
    pp = gpu_pp(8)
    assert len(pp.verify_range_proofs([], [])) == 0
    raw, com = _mk(pp, 200, 42)
    assert list(pp.verify_range_proofs([raw], [com])) == [0]


def test_staged_batch_reverifies(gpu_pp):
    pp = gpu_pp(16)
    proofs, coms = pp.prove_range_batch(list(range(1000, 1064)), [(i + 5).to_bytes(32, "big") for i in range(64)], 5)
    proofs[10] = proofs[11]
    b = pp.stage_range_proofs(proofs, coms)
    for _ in range(3):
        st = b.verify()
        assert int(st[10]) != 0 and int((st != 0).sum()) == 1
    b.close()


def test_reference_shaped_api(gpu_pp):
    import fts_gpu
    pp = gpu_pp(8)
    raw, com = _mk(pp, 115, 77)
    fts_gpu.RangeVerifier(pp, com).Verify(raw)
    raw2, _ = _mk(pp, 116, 78)
    with pytest.raises(fts_gpu.VerifyError) as e:
        fts_gpu.RangeVerifier(pp, com).Verify(raw2)
    assert str(e.value) == "invalid range proof"


@pytest.mark.parametrize("path", ["latency", "work"])
def test_full_batch_exact_intermediates_vs_cpu_batch(gpu_pp, pp_raw, oracle_pp, path):
    """BASELINE C2 at full size with EXACT intermediates: 4,096 rp64 proofs
    (1 % tampered in T1, an L_j or the IPA's a), every verdict, every com and
    every x0 on the device equal those of the independent CPU batch verifier
    (oracle/c/cpu_batch.c: its com / x0 pinned by the golden vectors, its
    failing proofs' verdicts from the reference-order restatement); on both
    com paths (latency: fixed-base groups + x*D; work: Horner + joint chain)"""
    from oracle import cref
    pp = gpu_pp(64) if path == "latency" else _work_path_pp(pp_raw, 64)
    n = 4096
    rng = random.Random(0xC2C2 + (path == "work"))
    vals = [rng.getrandbits(64) for _ in range(n)]
    bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(n)]
    proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=0xC2C2)
    for i in sorted(rng.sample(range(n), 41)):
        r = zkat.RangeProof.deserialize(proofs[i])
        kind = rng.randrange(3)
        if kind == 0:
            r.data.T1 = bn.g1_add(r.data.T1, bn.GEN)
        elif kind == 1:
            j = rng.randrange(6)
            r.ipa.L[j] = bn.g1_add(r.ipa.L[j], bn.GEN)
        else:
            r.ipa.Left = (r.ipa.Left + 1) % bn.R
        proofs[i] = r.serialize()
    st = pp.verify_range_proofs(proofs, coms)
    assert ("k_rp_fixed_all" in pp.last_timings()) == (path == "latency")
    cb = cref.CpuBatch(oracle_pp.with_bit_length(64), window_bits=10, threads=8)
    want, nfb, com_c, x0_c = cb.verify_ex(coms, proofs, threads=8)
    cb.close()
    assert [int(s) for s in st] == want
    assert 0 < sum(w != 0 for w in want) <= 41 and nfb > 0
    for i in range(n):
        v, com, _ = _intermediates(pp, i)
        assert com == com_c[i], i
        assert v[7] == int.from_bytes(x0_c[i], "big"), i
