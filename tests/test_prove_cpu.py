"""CPU checks of the device-prover host plumbing (no GPU): the packed
fts_action_witness array, and that the device entry points refuse a host-only
context (they must never fall back to the host prover)."""
import ctypes as C

import pytest


def test_witness_batch_packing():
    import fts_gpu
    acts = [(b"ABC", [1, 2], [b"a" * 32, b"b" * 32], [3], [b"c" * 32]),
            (b"", [], [], [7, 8], [b"d" * 32, b"e" * 32])]
    wb = fts_gpu.WitnessBatch(acts)
    for i, (t, iv, ib, ov, ob) in enumerate(acts):
        it = wb.items[i]
        assert it.type_len == len(t) and (not t or C.string_at(it.type, it.type_len) == t)
        assert it.n_in == len(iv) and it.n_out == len(ov)
        assert [C.c_uint64.from_address(it.in_values + 8 * k).value for k in range(it.n_in)] == iv
        assert [C.c_uint64.from_address(it.out_values + 8 * k).value for k in range(it.n_out)] == ov
        assert C.string_at(it.in_bfs, 32 * len(ib)) == b"".join(ib) if ib else True
        assert C.string_at(it.out_bfs, 32 * len(ob)) == b"".join(ob)


def test_device_provers_need_a_device(host_pp):
    import fts_gpu
    pp = host_pp(8)
    with pytest.raises(fts_gpu.FtsError):
        pp.prove_range_batch_gpu([1], [bytes(32)], seed=1)
    with pytest.raises(fts_gpu.FtsError):
        pp.prove_transfers_gpu([(b"A", [1], [bytes(32)], [1], [bytes(32)])], seed=1)
    with pytest.raises(fts_gpu.FtsError):
        pp.check_openings([(bytes(64), b"A", bytes(32), bytes(32))])


def test_secure_prover_randomness(host_pp, oracle_pp):
    """FTS_SEED_OS_RANDOM: fresh getrandom() key per call -> two proofs of the same
    witness differ in every random element, and both verify (C oracle,
    reference order); a seeded call stays reproducible (tests/bench mode)."""
    import fts_gpu
    from oracle import cref, zkat
    pp = host_pp(16)
    bf = (12345).to_bytes(32, "big")
    p1, c1 = pp.prove_range(777, bf, fts_gpu.FTS_SEED_OS_RANDOM)
    p2, c2 = pp.prove_range(777, bf, fts_gpu.FTS_SEED_OS_RANDOM)
    assert c1 == c2 and p1 != p2
    r1, r2 = zkat.RangeProof.deserialize(p1), zkat.RangeProof.deserialize(p2)
    assert r1.data.T1 != r2.data.T1 and r1.data.C != r2.data.C and r1.data.Tau != r2.data.Tau
    opp = oracle_pp.with_bit_length(16)
    assert cref.rp_verify_many(opp, [c1, c2], [p1, p2]) == [0, 0]
    b1, _ = pp.prove_range_batch([5, 6], [bf, bf], fts_gpu.FTS_SEED_OS_RANDOM)
    b2, _ = pp.prove_range_batch([5, 6], [bf, bf], fts_gpu.FTS_SEED_OS_RANDOM)
    assert b1[0] != b2[0] and b1[1] != b2[1]
    assert pp.prove_range(777, bf, 9)[0] == pp.prove_range(777, bf, 9)[0]
    t = pp.prove_transfer(b"ABC", [3, 4], [bf, bf], [5, 2], [bf, bf], fts_gpu.FTS_SEED_OS_RANDOM)
    ins = [pp.token_commit(b"ABC", v, bf) for v in (3, 4)]
    outs = [pp.token_commit(b"ABC", v, bf) for v in (5, 2)]
    assert cref.action_verify_many(opp, [("transfer", ins, outs, t)]) == [(0, -1)]
