"""GPU: batched range-proof prover (fts_rp_prove_batch_gpu).

rangeProver.Prove (rp/bulletproof.go:209-249, :336-466) and the IPA prover
(rp/ipa.go:158-186, :267-322) on the device.  Parity: the device proofs are
byte-identical to the library's host prover for the same seeds (the host
prover is itself pinned by the oracle: tests/test_lib_cpu.py verifies its
proofs with the reference-order oracle verifier), they are accepted by the
oracle's verifier and by the device verifier, and out-of-range values give
the same (rejected) proofs as on the host."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _inputs(n, bits, seed):
    rng = random.Random(seed)
    vals = [0, (1 << bits) - 1, 1, 1 << (bits - 1)] + [rng.randrange(1 << bits) for _ in range(n - 4)]
    bfs = [rng.randrange(1 << 250).to_bytes(32, "big") for _ in range(n)]
    return vals, bfs


@pytest.mark.parametrize("bits", [8, 32, 64])
def test_device_prover_matches_host_prover(gpu_pp, bits):
    pp = gpu_pp(bits)
    vals, bfs = _inputs(24, bits, bits)
    dev, dcoms = pp.prove_range_batch_gpu(vals, bfs, seed=1000 + bits)
    host, hcoms = pp.prove_range_batch(vals, bfs, seed=1000 + bits)
    assert dcoms == hcoms
    assert dev == host
    assert [int(s) for s in pp.verify_range_proofs(dev, dcoms)] == [0] * len(vals)


def test_device_proofs_accepted_by_oracle(gpu_pp, oracle_pp):
    from oracle import bn254 as bn, zkat
    pp = gpu_pp(64)
    vals, bfs = _inputs(4, 64, 7)
    proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=77)
    for p, c in zip(proofs, coms):
        rp = zkat.RangeProof.deserialize(p)
        assert zkat.rp_verify(bn.g1_from_bytes(c), oracle_pp.ped[1:], oracle_pp.left, oracle_pp.right,
                              oracle_pp.P, oracle_pp.Q, 6, 64, rp) is None


def test_device_prover_out_of_range_value(gpu_pp):
    """value >= 2^bits: the reference prover still outputs a proof, which fails"""
    import fts_gpu as F
    pp = gpu_pp(32)
    vals = [1 << 32, (1 << 40) + 5, 3]
    bfs = [(9 + i).to_bytes(32, "big") for i in range(3)]
    dev, coms = pp.prove_range_batch_gpu(vals, bfs, seed=5)
    host, _ = pp.prove_range_batch(vals, bfs, seed=5)
    assert dev == host
    st = [int(s) for s in pp.verify_range_proofs(dev, coms)]
    assert st[2] == F.FTS_OK and st[0] != F.FTS_OK and st[1] != F.FTS_OK


def test_device_prover_large_batch_verifies(gpu_pp):
    """20,000 proofs (two device passes) -> all accepted by the device verifier; a sample
    matches the host prover"""
    pp = gpu_pp(64)
    n = 20000
    rng = random.Random(3)
    vals = [rng.randrange(1 << 64) for _ in range(n)]
    bfs = [rng.randrange(1 << 250).to_bytes(32, "big") for _ in range(n)]
    proofs, coms = pp.prove_range_batch_gpu(vals, bfs, seed=90000)
    st = pp.verify_range_proofs(proofs, coms)
    assert int((st != 0).sum()) == 0
    idx = [0, 16383, 16384, n - 1]
    # the host batch seeds proof j with seed + j: re-prove each sampled proof with its own seed
    for i in idx:
        h, hc = pp.prove_range_batch([vals[i]], [bfs[i]], seed=90000 + i)
        assert h[0] == proofs[i] and hc[0] == coms[i]


def _bf(rng):
    return rng.randrange(1 << 250).to_bytes(32, "big")


def test_device_transfer_prover_matches_host(gpu_pp):
    """TypeAndSum + range proofs on the device == host prove_transfer (1-in/1-out: no range
    proofs, transfer.go:85-87); the device verifier accepts them"""
    pp = gpu_pp(64)
    rng = random.Random(11)
    trs = []
    for nin, nout in [(2, 2), (1, 1), (1, 2), (3, 1), (2, 3)]:
        iv = [rng.randrange(1 << 40) for _ in range(nin)]
        tot = sum(iv)
        ov = [rng.randrange(tot + 1) for _ in range(nout - 1)] if nout > 1 else []
        ov = [min(v, tot - sum(ov[:i])) for i, v in enumerate(ov)]
        ov.append(tot - sum(ov))
        trs.append((b"ABC" if nin % 2 else b"USD", iv, [_bf(rng) for _ in iv], ov, [_bf(rng) for _ in ov]))
    dev = pp.prove_transfers_gpu(trs, seed=500)
    for i, (t, iv, ib, ov, ob) in enumerate(trs):
        assert dev[i] == pp.prove_transfer(t, iv, ib, ov, ob, seed=500 + i), i
    items = [([pp.token_commit(t, v, b) for v, b in zip(iv, ib)], [pp.token_commit(t, v, b) for v, b in zip(ov, ob)],
              dev[i]) for i, (t, iv, ib, ov, ob) in enumerate(trs)]
    st, fi = pp.verify_transfers(items)
    assert [int(x) for x in st] == [0] * len(trs)


def test_device_issue_prover_matches_host(gpu_pp, oracle_pp):
    import fts_gpu as F
    from oracle import bn254 as bn, zkat
    pp = gpu_pp(32)
    rng = random.Random(12)
    iss = [(b"ABC", [rng.randrange(1 << 32) for _ in range(m)], [_bf(rng) for _ in range(m)]) for m in (1, 4, 16)]
    dev = pp.prove_issues_gpu(iss, seed=600)
    for i, (t, v, b) in enumerate(iss):
        assert dev[i] == pp.prove_issue(t, v, b, seed=600 + i), i
    t, v, b = iss[1]
    toks = [pp.token_commit(t, x, y) for x, y in zip(v, b)]
    F.IssueVerifier(toks, pp).Verify(dev[1])
    opp = oracle_pp.with_bit_length(32)
    err, _ = zkat.issue_verify(opp, [bn.g1_from_bytes(x) for x in toks], dev[1])
    assert err is None
