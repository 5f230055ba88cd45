"""Multi-GPU exchange step on CPU: world-size-2 `gloo` process groups run the
same helpers bench.py uses over RCCL (fts_gpu.dist): the all-gather of
per-rank verdict bitmaps, max-over-ranks timing, summed accept counts, and
disjoint per-rank input shards (no collective on the data path)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _n_of(rank, n):
    return n + 13 * rank  # uneven shards: ranks hold different proof counts


def _verdicts(rank, n):
    n = _n_of(rank, n)
    rng = np.random.default_rng(1000 + rank)
    st = np.zeros(n, dtype=np.int32)
    bad = rng.choice(n, size=3 + rank, replace=False)
    st[bad] = 3 + rank  # rank-specific rejections
    return st


def _worker(rank, world, port, n, q):
    sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # the exchange helpers only need torch.distributed; keep libfts_gpu unloaded
    import importlib.util

    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location(
        "fts_dist", os.path.join(ROOT, "fabric-token-sdk_amd", "fts_gpu", "dist.py"))
    fdist = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fdist)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = _verdicts(rank, n)
        bitmap = fdist.allgather_verdicts(dist, st)
        tmax = fdist.reduce_scalar(dist, 1.5 + rank, "max")
        oks = fdist.reduce_scalar(dist, int((st == 0).sum()), "sum")
        seeds = [fdist.shard_seed(0xF7A50002, rank, s) for s in range(4)]
        q.put((rank, bitmap.tolist(), tmax, oks, seeds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [4096, 37])
def test_gloo_world2_verdict_exchange(n):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.concatenate([_verdicts(r, n) == 0 for r in range(2)]).tolist()
    for rank, bitmap, tmax, oks, seeds in res:
        assert bitmap == expect                                # every rank holds every shard's verdicts, in order
        assert len(bitmap) == _n_of(0, n) + _n_of(1, n)        # one entry per proof (no packing pad)
        assert tmax == 2.5                                     # max over ranks (bench's job time)
        assert oks == sum(int((_verdicts(r, n) == 0).sum()) for r in range(2))
    assert not set(res[0][4]) & set(res[1][4])                # disjoint input shards
