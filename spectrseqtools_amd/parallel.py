"""Multi-GPU layer: one process per GPU, spectra sharded by rank, results
gathered to rank 0 over RCCL (torch.distributed backend "nccl" on ROCm) /
gloo on CPU.

The path partitions cleanly: every is_valid / explain query depends only on
its own spectrum and the read-only table, so each rank builds its own table
replica (milliseconds on the GPU) and processes its own spectra.  The only
exchange step is delivering the compact per-query results (status, count,
candidate payload) to the rank that drives the Python pipeline.  RCCL has no
gatherv: sizes are agreed once (all_gather of lengths), then one padded
torch.distributed.gather moves the bytes (send/recv over xGMI).
"""
import os

import numpy as np


def dist_env():
    """(rank, world_size, local_rank) from torchrun's environment."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_range(n_items, rank, world):
    """Contiguous, balanced [start, stop) of n_items for this rank."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_by_weight(weights, world):
    """Contiguous split of items with the given costs into `world` ranges of
    near-equal total cost (spectra balanced by query count)."""
    w = np.asarray(weights, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(len(w))
    cuts = np.maximum.accumulate(np.asarray(cuts))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


class Gatherer:
    """Gather one flat uint8 buffer per rank to rank 0.

    agree() fixes the per-rank byte counts (one all_gather of int64 sizes);
    gather() then moves the bytes with a single padded dist.gather.  Works
    for the nccl (device tensors) and gloo (host tensors) backends."""

    def __init__(self, dist, device):
        self.dist = dist
        self.device = device
        self.sizes = None
        self.recv = None

    def agree(self, nbytes):
        import torch

        t = torch.tensor([int(nbytes)], dtype=torch.int64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(out, t)
        self.sizes = [int(x.item()) for x in out]
        self.max = max(self.sizes) if self.sizes else 0
        if self.dist.get_rank() == 0:
            self.recv = [torch.empty(self.max, dtype=torch.uint8, device=self.device)
                         for _ in range(self.dist.get_world_size())]
        return self.sizes

    def gather(self, buf):
        """buf: uint8 tensor of exactly this rank's agreed size (padded here).
        Returns the per-rank buffers (trimmed) on rank 0, None elsewhere."""
        import torch

        rank = self.dist.get_rank()
        if buf.numel() < self.max:
            pad = torch.zeros(self.max - buf.numel(), dtype=torch.uint8, device=buf.device)
            buf = torch.cat([buf, pad])
        if rank == 0:
            self.dist.gather(buf, gather_list=self.recv, dst=0)
            return [r[:n] for r, n in zip(self.recv, self.sizes)]
        self.dist.gather(buf, dst=0)
        return None


def device_bytes(ptr, nbytes, device):
    """Zero-copy uint8 torch view of an engine device buffer."""
    import torch

    class _Iface:
        __cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                    "version": 3, "strides": None}

    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8, device=device)
    return torch.as_tensor(_Iface(), device=device)
