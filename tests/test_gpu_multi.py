"""GPU: multi-device contexts (fts_ctx_create_devices / _mask; SURVEY §8b device_mask,
§8e).  A one-device mask must give exactly the single-device context's verdicts; a
context of two shards on the same GPU exercises the split / concurrent run / merge
path of every sharded entry point on a one-GPU box (the driver's 8-GPU node runs
the same code with eight distinct devices)."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "transfer_golden.json")) as f:
    TRANSFERS = [c for c in json.load(f) if c["bits"] == 16]
with open(os.path.join(GOLDEN, "rp_golden.json")) as f:
    RPS = [c for c in json.load(f) if c["bits"] == 16]

_MULTI = {}


def _multi(pp_raw, devices):
    import fts_gpu
    key = tuple(devices)
    if key not in _MULTI:
        _MULTI[key] = fts_gpu.PublicParams(pp_raw, bit_length=16, devices=list(devices))
    return _MULTI[key]


def _transfer_items(pp, n, seed):
    """n 2-in/2-out 16-bit transfers, every 5th with a wrong sum, every 7th with swapped range proofs"""
    from oracle import der
    rng = random.Random(seed)
    T, items = b"ABC", []
    for i in range(n):
        a, b = rng.randrange(1 << 14), rng.randrange(1 << 14)
        c = rng.randrange(a + b + 1)
        outs = [c, a + b - c + (1 if i % 5 == 3 else 0)]
        ib = [rng.randrange(1, 1 << 200).to_bytes(32, "big") for _ in range(2)]
        ob = [rng.randrange(1, 1 << 200).to_bytes(32, "big") for _ in range(2)]
        proof = pp.prove_transfer(T, [a, b], ib, [c, a + b - c], ob, 1000 + i)
        if i % 7 == 6:
            t, rc = der.unmarshal_values(proof)
            rps = der.unmarshal_values(der.unmarshal_values(rc)[0])
            proof = der.values([t, der.values([der.values([rps[1], rps[0]])])])
        items.append(([pp.token_commit(T, v, x) for v, x in zip([a, b], ib)],
                      [pp.token_commit(T, v, x) for v, x in zip(outs, ob)], proof))
    return items


def test_one_device_mask_equals_single_context(gpu_pp, pp_raw):
    import fts_gpu
    single = gpu_pp(16)
    multi = _multi(pp_raw, [0])
    assert multi.devices == [0] and single.devices == [0]
    items = [([bytes.fromhex(h) for h in c["inputs"]], [bytes.fromhex(h) for h in c["outputs"]],
              bytes.fromhex(c["proof"])) for c in TRANSFERS]
    s1, f1 = single.verify_transfers(items)
    s2, f2 = multi.verify_transfers(items)
    assert (s1 == s2).all() and (f1 == f2).all()
    assert [fts_gpu.transfer_message(int(s), int(i)) for s, i in zip(s2, f2)] == [c["expect"] for c in TRANSFERS]


def test_two_shards_every_entry_point(gpu_pp, pp_raw):
    """devices [0, 0]: each batch is split in two, run concurrently, merged in caller order"""
    single = gpu_pp(16)
    multi = _multi(pp_raw, [0, 0])
    assert multi.devices == [0, 0]
    # standalone range proofs (golden, tiled so both shards get proofs of every class)
    proofs = [bytes.fromhex(c["proof"]) for c in RPS] * 3
    coms = [bytes.fromhex(c["commitment"]) for c in RPS] * 3
    assert (multi.verify_range_proofs(proofs, coms) == single.verify_range_proofs(proofs, coms)).all()
    # transfers with failures spread over both shards
    items = _transfer_items(single, 23, 5)
    s1, f1 = single.verify_transfers(items)
    s2, f2 = multi.verify_transfers(items)
    assert (s1 == s2).all() and (f1 == f2).all() and (s1 != 0).sum() >= 5
    # mixed transfers + issues in one call
    T = b"USD"
    issues = []
    for i in range(6):
        vals = [(i * 31 + j * 7) % (1 << 16) for j in range(4)]
        bfs = [(77 + i * 4 + j).to_bytes(32, "big") for j in range(4)]
        toks = [single.token_commit(T, v, x) for v, x in zip(vals, bfs)]
        if i == 4:
            toks[2] = single.token_commit(T, vals[2] + 1, bfs[2])
        issues.append((toks, single.prove_issue(T, vals, bfs, 50 + i)))
    a1 = single.verify_actions(items, issues)
    a2 = multi.verify_actions(items, issues)
    for x, y in zip(a1, a2):
        assert (x == y).all()
    # staged batches
    st = multi.stage_range_proofs(proofs, coms)
    assert (st.verify() == single.verify_range_proofs(proofs, coms)).all()
    st.close()
    # MSM: partial points of the two devices combined on the host
    rng = random.Random(9)
    pts, scs = [], []
    for i in range(300):
        pts.append(single.token_commit(b"M", i, (i + 1).to_bytes(32, "big")))
        scs.append(rng.randrange(1 << 254).to_bytes(32, "big"))
    assert multi.msm(pts, scs) == single.msm(pts, scs)
    # token openings
    ops = [(single.token_commit(T, v, (v + 9).to_bytes(32, "big")), T, v.to_bytes(32, "big"),
            (v + 9 + (1 if v % 4 == 0 else 0)).to_bytes(32, "big")) for v in range(41)]
    assert (multi.check_openings(ops) == single.check_openings(ops)).all()
    assert int((multi.check_openings(ops) != 0).sum()) == 11
    assert np.array_equal(multi.check_openings(ops[:1]), single.check_openings(ops[:1]))
