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
