"""GPU: BASELINE config C2 at full size (4,096 standalone 64-bit range proofs
in one batch) through size-independent properties: every honest proof is
accepted, exactly the tampered positions are rejected with the reference's
error class, and re-verifying the staged batch is idempotent."""
import random

import pytest

from oracle import bn254 as bn, zkat

pytestmark = pytest.mark.gpu


def test_full_batch_4096_rp64(gpu_pp):
    pp = gpu_pp(64)
    n = 4096
    rng = random.Random(0xF7A50002)
    vals = [rng.getrandbits(64) for _ in range(n)]
    bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(n)]
    proofs, coms = pp.prove_range_batch(vals, bfs, seed=0xF7A50002)
    b = pp.stage_range_proofs(proofs, coms)
    st = b.verify()
    assert int((st != 0).sum()) == 0
    # 1% tampered: random T1 (-> invalid range proof) or L_j (-> invalid IPA)
    bad = sorted(rng.sample(range(n), 41))
    kinds = {}
    for i in bad:
        r = zkat.RangeProof.deserialize(proofs[i])
        if rng.random() < 0.5:
            r.data.T1 = bn.g1_add(r.data.T1, bn.GEN)
            kinds[i] = 3
        else:
            j = rng.randrange(6)
            r.ipa.L[j] = bn.g1_add(r.ipa.L[j], bn.GEN)
            kinds[i] = 6
        proofs[i] = r.serialize()
    b2 = pp.stage_range_proofs(proofs, coms)
    st2 = b2.verify()
    assert {i: int(st2[i]) for i in range(n) if st2[i] != 0} == kinds
    assert (b2.verify() == st2).all()
    b.close()
    b2.close()


def test_concurrent_lanes_rp32(gpu_pp):
    """Concurrent fts_rp_batch_verify calls on different staged batches run on
    different device lanes (stream pairs + workspaces): every batch must still
    get exactly its own verdicts (tampered positions differ per batch)."""
    import threading

    pp = gpu_pp(32)
    rng = random.Random(0xF7A5C0DE)
    batches, expect = [], []
    for t in range(4):
        m = 96
        vals = [rng.getrandbits(32) for _ in range(m)]
        bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(m)]
        proofs, coms = pp.prove_range_batch(vals, bfs, seed=1000 + t)
        bad = set(rng.sample(range(m), 3 + t))
        for i in bad:
            r = zkat.RangeProof.deserialize(proofs[i])
            r.data.T2 = bn.g1_add(r.data.T2, bn.GEN)
            proofs[i] = r.serialize()
        batches.append(pp.stage_range_proofs(proofs, coms))
        expect.append([3 if i in bad else 0 for i in range(m)])
    out = [[] for _ in batches]

    def work(t):
        for _ in range(3):
            out[t].append([int(s) for s in batches[t].verify()])

    th = [threading.Thread(target=work, args=(t,)) for t in range(len(batches))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for t in range(len(batches)):
        assert len(out[t]) == 3
        for st in out[t]:
            assert st == expect[t]
        batches[t].close()


def test_coalesced_batches_keep_their_verdicts(pp_raw):
    """With ONE device lane, batches submitted concurrently are coalesced into
    shared device passes (fts_rp_batch_verify's dispatcher).  Each caller must
    still get exactly its own per-proof verdicts, including the per-proof
    fallback (tampered proofs make the merged combination fail)."""
    import os
    import threading

    import fts_gpu

    old = os.environ.get("FTS_LANES")
    os.environ["FTS_LANES"] = "1"
    try:
        pp = fts_gpu.PublicParams(pp_raw, bit_length=16, device=0)
    finally:
        if old is None:
            del os.environ["FTS_LANES"]
        else:
            os.environ["FTS_LANES"] = old
    rng = random.Random(0xC0A1E5CE)
    sizes = [1, 7, 64, 200, 33, 128, 5, 90]
    batches, expect = [], []
    for t, m in enumerate(sizes):
        vals = [rng.getrandbits(16) for _ in range(m)]
        bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(m)]
        proofs, coms = pp.prove_range_batch(vals, bfs, seed=5000 + t)
        exp = [0] * m
        if t % 2 == 1:  # odd batches carry tampered proofs of both classes
            for i in rng.sample(range(m), min(m, 2 + t // 2)):
                r = zkat.RangeProof.deserialize(proofs[i])
                if rng.random() < 0.5:
                    r.data.T1 = bn.g1_add(r.data.T1, bn.GEN)
                    exp[i] = 3
                else:
                    r.ipa.R[rng.randrange(4)] = bn.g1_add(r.ipa.R[0], bn.GEN)
                    exp[i] = 6
                proofs[i] = r.serialize()
        batches.append(pp.stage_range_proofs(proofs, coms))
        expect.append(exp)
    out = [[] for _ in batches]
    merged = []

    def work(t):
        for _ in range(4):
            out[t].append([int(s) for s in batches[t].verify()])
            merged.append(batches[t].merged())

    th = [threading.Thread(target=work, args=(t,)) for t in range(len(batches))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for t in range(len(batches)):
        assert len(out[t]) == 4
        for st in out[t]:
            assert st == expect[t], t
    assert max(merged) > 1, merged  # the dispatcher did merge batches
    for b in batches:
        b.close()
    pp.close()


def test_one_bad_proof_in_coalesced_pass_group_test(pp_raw):
    """SURVEY Appendix B fallback: one tampered proof inside a coalesced pass of 8
    caller batches.  The failed batch check is narrowed by group tests (groups never
    straddle two caller batches) so only a handful of proofs -- all of the bad
    proof's own batch -- get the per-proof final equations; every verdict equals
    the reference's (rangecorrectness.go:141-160)."""
    import os
    import threading

    import fts_gpu

    old = os.environ.get("FTS_LANES")
    os.environ["FTS_LANES"] = "1"
    try:
        pp = fts_gpu.PublicParams(pp_raw, bit_length=16, device=0)
    finally:
        if old is None:
            del os.environ["FTS_LANES"]
        else:
            os.environ["FTS_LANES"] = old
    rng = random.Random(0xB15EC7)
    m, nb, bad_batch, bad_idx = 512, 8, 3, 333
    batches, expect = [], []
    for t in range(nb):
        vals = [rng.getrandbits(16) for _ in range(m)]
        bfs = [rng.randrange(bn.R).to_bytes(32, "big") for _ in range(m)]
        proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=7000 + 1000 * t)
        exp = [0] * m
        if t == bad_batch:
            r = zkat.RangeProof.deserialize(proofs[bad_idx])
            r.ipa.L[1] = bn.g1_add(r.ipa.L[1], bn.GEN)
            proofs[bad_idx] = r.serialize()
            exp[bad_idx] = 6
        batches.append(pp.stage_range_proofs(proofs, coms))
        expect.append(exp)
    # occupy the single lane so the 8 submissions queue up and coalesce
    blocker = batches[0]
    out, merged, tim = [None] * nb, [0] * nb, [None] * nb

    def work(t):
        out[t] = [int(s) for s in batches[t].verify()]
        merged[t] = batches[t].merged()
        tim[t] = batches[t].timings()

    th = [threading.Thread(target=blocker.verify)] + [threading.Thread(target=work, args=(t,)) for t in range(nb)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for t in range(nb):
        assert out[t] == expect[t], t
    assert merged[bad_batch] > 1, merged
    tb = tim[bad_batch]
    assert "fb:k_rlc_group_final" in tb and "fb:k_rp_terms_fixed" in tb, sorted(tb)
    per_proof = tb["fb:k_rp_terms_fixed"][1] / ((3 + 2 * 16) * 15 * 11 * 136)
    # the bad proof's round-1 group (256 proofs of its own batch), not the pass (4,096)
    assert 1 <= round(per_proof) <= 256, per_proof
    for b in batches:
        b.close()
    pp.close()
