"""Multi-GPU exchange step: proofs shard naturally, one process
per GPU verifies its own shard with no collective on the data path; the only
exchange is an all-gather of per-GPU verdict bitmaps (B/8 bytes per batch)
plus scalar reductions for the job's timing and counts.

Works with the "nccl" backend (RCCL over xGMI, device tensors) and with
"gloo" (CPU tensors; used by the world-size-2 tests on CPU)."""
import numpy as np


def _dev(dist):
    import torch
    return torch.device("cuda") if dist.get_backend() == "nccl" else torch.device("cpu")


def allgather_verdicts(dist, status):
    """status: this rank's per-proof verdicts (np.int32, 0 = accepted; any length,
    ranks may differ) -> np.bool_ array of accepted flags of ALL ranks' proofs,
    concatenated in rank order (one entry per proof, no padding).

    Two collectives: the per-rank counts first, then the bit-packed verdicts padded
    to the largest rank's packed size (all_gather_into_tensor needs equal sizes);
    each rank's block is unpacked and trimmed to its true count."""
    import torch
    dev = _dev(dist)
    acc = np.asarray(status) == 0
    world = dist.get_world_size()
    cnt = torch.tensor([acc.size], dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, cnt)
    counts = [int(c) for c in counts.cpu()]
    width = max(1, (max(counts) + 7) // 8)
    packed = np.zeros(width, dtype=np.uint8)
    pb = np.packbits(acc)
    packed[:pb.size] = pb
    bits = torch.from_numpy(packed).to(dev)
    out = torch.empty(world * width, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, bits)
    blocks = out.cpu().numpy().reshape(world, width)
    return np.concatenate([np.unpackbits(blocks[r])[:counts[r]].astype(bool) for r in range(world)])


def allgather_status(dist, values):
    """values: this rank's int32 array (e.g. fts_status per action, or interleaved
    (status, fail_index) pairs; ranks may hold different lengths) -> the int32
    concatenation of ALL ranks' arrays in rank order.  Same two-collective shape
    as allgather_verdicts (counts, then equal-size padded blocks), for endorsers
    that need the error class and failing index of every item, not only the bit."""
    import torch
    dev = _dev(dist)
    v = np.ascontiguousarray(np.asarray(values, dtype=np.int32).ravel())
    world = dist.get_world_size()
    cnt = torch.tensor([v.size], dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, cnt)
    counts = [int(c) for c in counts.cpu()]
    width = max(1, max(counts))
    pad = np.zeros(width, dtype=np.int32)
    pad[:v.size] = v
    out = torch.empty(world * width, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(out, torch.from_numpy(pad).to(dev))
    blocks = out.cpu().numpy().reshape(world, width)
    return np.concatenate([blocks[r][:counts[r]] for r in range(world)])


def reduce_scalar(dist, x, op="max"):
    """max/sum of a Python number over ranks"""
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def shard_seed(base, rank, slot=0):
    """seed of the synthetic inputs of (rank, slot): disjoint shards per rank"""
    return base + 7919 * rank + 104729 * slot
