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
    """status: this rank's per-proof verdicts (np.int32, 0 = accepted) ->
    np.uint8 bitmap of accepted proofs, all ranks concatenated in rank order"""
    import torch
    bits = torch.from_numpy(np.packbits(np.asarray(status) == 0)).to(_dev(dist))
    out = torch.empty(dist.get_world_size() * bits.numel(), dtype=torch.uint8, device=bits.device)
    dist.all_gather_into_tensor(out, bits)
    return out.cpu().numpy()


def reduce_scalar(dist, x, op="max"):
    """max/sum of a Python number over ranks"""
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def shard_seed(base, rank, slot=0):
    """seed of the synthetic inputs of (rank, slot): disjoint shards per rank"""
    return base + 7919 * rank + 104729 * slot
