"""GPU: standalone BN254 G1 MSM (fts_msm_g1, BASELINE config C3) against the
oracle's sum of (k mod r)·P (oracle/bn254.py g1_msm = mathlib G1.Mul + Add,
the value gnark-crypto's MultiExp returns).  Small sizes are compared point
by point; the 2^16-point case is checked through a size-independent
identity: with P_i = (i+1)·G, sum k_i P_i = (sum k_i (i+1) mod r)·G."""
import random

import pytest

from oracle import bn254 as bn

pytestmark = pytest.mark.gpu


def _pts(points):
    return b"".join(bn.g1_bytes(p) for p in points)


def _scs(scalars):
    return b"".join((k % (1 << 256)).to_bytes(32, "big") for k in scalars)


@pytest.mark.parametrize("n", [1, 2, 17, 300])
def test_msm_random_matches_oracle(gpu_pp, n):
    pp = gpu_pp(64)
    rng = random.Random(0xC3000 + n)
    points = [bn.g1_mul(bn.GEN, rng.randrange(1, bn.R)) for _ in range(n)]
    # full 256-bit scalars: some exceed r (used mod r, as G1.Mul does)
    scalars = [rng.getrandbits(256) for _ in range(n)]
    got = pp.msm(_pts(points), _scs(scalars))
    assert got == bn.g1_bytes(bn.g1_msm(points, scalars))


def test_msm_edge_cases(gpu_pp):
    pp = gpu_pp(64)
    rng = random.Random(0xC3E)
    P = bn.g1_mul(bn.GEN, rng.randrange(1, bn.R))
    Q = bn.g1_mul(bn.GEN, rng.randrange(1, bn.R))
    k = rng.randrange(bn.R)
    cases = [
        ([P], [0]),                                   # zero scalar -> identity
        ([P], [bn.R]),                                # r = 0 mod r -> identity
        ([P, bn.g1_neg(P)], [k, k]),                  # P + (-P) -> identity
        ([P, P], [k, bn.R - k]),                      # k P + (r - k) P -> identity
        ([P, P, P], [1, 1, 1]),                       # same bucket, doubling inside the bucket sum
        ([None, P], [k, 5]),                          # identity point (64 zero bytes)
        ([P, Q], [bn.R - 1, (1 << 256) - 1]),         # extreme scalars
        ([P] * 64, list(range(64))),                  # many points in few buckets
    ]
    for points, scalars in cases:
        got = pp.msm(_pts(points), _scs(scalars))
        assert got == bn.g1_bytes(bn.g1_msm([p for p in points], scalars)), (points, scalars)


def test_msm_rejects_bad_point(gpu_pp):
    import fts_gpu

    pp = gpu_pp(64)
    bad = bytearray(bn.g1_bytes(bn.GEN))
    bad[63] ^= 1  # off the curve
    with pytest.raises(fts_gpu.FtsError):
        pp.msm(bytes(bad) + bn.g1_bytes(bn.GEN), _scs([3, 4]))


def test_msm_2p16_linear_identity(gpu_pp):
    pp = gpu_pp(64)
    n = 1 << 16
    rng = random.Random(0xF7A50003)
    # P_i = (i+1) G by successive additions (Jacobian, one normalisation each)
    points, acc = [], None
    for _ in range(n):
        acc = bn.g1_add(acc, bn.GEN)
        points.append(acc)
    scalars = [rng.randrange(bn.R) for _ in range(n)]
    expect = bn.g1_mul(bn.GEN, sum(k * (i + 1) for i, k in enumerate(scalars)) % bn.R)
    st = pp.stage_msm(_pts(points), _scs(scalars))
    got = st.run()
    assert got == bn.g1_bytes(expect)
    assert st.run() == got  # idempotent re-run on the staged inputs
    st.close()


def test_msm_2p20_linearity_and_identity(gpu_pp):
    """BASELINE config C3 at the top of its range used by the tests (2^20 points):
    MSM(P, a) + MSM(P, b) == MSM(P, a + b mod r) (linearity, three device MSMs),
    the closed form sum k_i (i mod 2^16 + 1) G for P_i = (i mod 2^16 + 1) G, and a
    300-term slice of the same points against the oracle term by term."""
    pp = gpu_pp(64)
    n, m = 1 << 20, 1 << 16
    rng = random.Random(0xC3020)
    base, acc = [], None
    for _ in range(m):
        acc = bn.g1_add(acc, bn.GEN)
        base.append(acc)
    pts = _pts(base) * (n // m)
    a = [rng.randrange(bn.R) for _ in range(n)]
    b = [rng.randrange(bn.R) for _ in range(n)]
    ab = [(x + y) % bn.R for x, y in zip(a, b)]
    ra, rb, rab = (bytes(pp.msm(pts, _scs(s))) for s in (a, b, ab))
    assert bn.g1_bytes(bn.g1_add(bn.g1_from_bytes(ra), bn.g1_from_bytes(rb))) == rab
    expect = bn.g1_mul(bn.GEN, sum(k * (i % m + 1) for i, k in enumerate(a)) % bn.R)
    assert ra == bn.g1_bytes(expect)
    lo = rng.randrange(n - 300)
    sl = slice(lo, lo + 300)
    got = pp.msm(pts[64 * lo:64 * (lo + 300)], _scs(a[sl]))
    assert got == bn.g1_bytes(bn.g1_msm([base[i % m] for i in range(lo, lo + 300)], a[sl]))


@pytest.mark.parametrize("log", [8, 18, 22])
def test_msm_distinct_device_points_closed_form(gpu_pp, oracle_pp, log):
    """config C3 as SURVEY §8(d) specifies it: 2^log DISTINCT points k_i ped1 made on
    the device (fts_msm_stage_multiples), scalars above r included (used mod r):
    sum s_i k_i ped1 = (sum s_i k_i mod r) ped1; at 2^8 the points are also compared
    with the oracle's through the host-staged MSM of the same points"""
    pp = gpu_pp(64)
    rng = random.Random(0xC3D0 + log)
    n = 1 << log
    ks = [rng.getrandbits(256) for _ in range(n)]
    ss = [rng.getrandbits(256) for _ in range(n)]
    st = pp.stage_msm_multiples(_scs(ks), _scs(ss))
    ped1 = oracle_pp.ped[1]
    want = bn.g1_bytes(bn.g1_mul(ped1, sum(s * k for s, k in zip(ss, ks)) % bn.R))
    assert st.run() == want
    assert st.run() == want  # re-run on the resident inputs
    # the staged points are the distinct k_i ped1 (fts_msm_points; a sample incl. both ends)
    for i in sorted({0, n - 1} | {rng.randrange(n) for _ in range(6)}):
        assert st.points(i, 1) == bn.g1_bytes(bn.g1_mul(ped1, ks[i] % bn.R)), i
    st.close()
    if log == 8:
        pts = [bn.g1_mul(ped1, k % bn.R) for k in ks]
        assert pp.msm(_pts(pts), _scs(ss)) == want


def test_msm_two_level_sort_adversarial_2p18(gpu_pp):
    """The two-level counting sort (msm.hip k_rs_*: the sort of the batch check's
    MSM and of standalone MSMs, round 5) on adversarial inputs: one scalar
    repeated by an eighth of the points (one bucket per window holds 32k entries,
    so one partition block sorts them all), zero scalars, r - 1 and scalars >= r
    (used mod r), identity points, and -P right after +P with the same scalar
    (the pair cancels); closed form sum s_i c_i G with P_i = c_i G"""
    pp = gpu_pp(64)
    n, m = 1 << 18, 1 << 16
    rng = random.Random(0x15A0)
    base, acc = [], None
    for _ in range(m):
        acc = bn.g1_add(acc, bn.GEN)
        base.append(acc)
    k_rep = rng.randrange(bn.R)
    pts, scs, total = [], [], 0
    for i in range(n):
        c = i % m + 1
        kind = i % 8
        if kind == 4 and i % 64 == 4:
            pts.append(None)  # identity point (64 zero bytes): contributes nothing
            scs.append(rng.randrange(bn.R))
            continue
        if kind == 5 and pts[-1] is not None:  # -P_{i-1} with P_{i-1}'s scalar
            c = -((i - 1) % m + 1)
            pts.append(bn.g1_neg(base[(i - 1) % m]))
            scs.append(scs[-1])
        else:
            s = {0: k_rep, 1: 0, 2: bn.R - 1, 3: rng.randrange(bn.R, 1 << 256)}.get(kind, rng.randrange(bn.R))
            pts.append(base[i % m])
            scs.append(s)
        total += (scs[-1] % bn.R) * c
    want = bn.g1_bytes(bn.g1_mul(bn.GEN, total % bn.R))
    st = pp.stage_msm(_pts(pts), _scs(scs))
    assert st.run() == want
    assert "k_rs_part" in st.timings() and "k_msm_digits" not in st.timings(), sorted(st.timings())
    st.close()
