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

Wire format of one rank's result (wire_pack / wire_unpack): a 32-B header
{u64 n_valid, n_explain, n_hits, payload_bytes}, the is_valid bytes, the
explain status bytes, the dense hit list (16-B records {u32 query, u32 count,
u64 word}: word = the candidates' payload offset (SOME) or the exact count
(OVERFLOW / ABORTED), include/sst.h sst_result_hit_list) and the dense
payload ([k][row_0..row_{k-1}] per candidate).  decode_hits turns it back
into per-query counts / offsets.
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
            self.last = [r[:n] for r, n in zip(self.recv, self.sizes)]
            return self.last
        self.dist.gather(buf, dst=0)
        self.last = None
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


WIRE_HEADER = 32
SST_SOME = 2


def wire_pack(valid, status, hits, payload):
    """One rank's result as a flat uint8 tensor (same device as the parts):
    header, is_valid bytes, status bytes, hit records, payload.  The parts
    are uint8 tensors (views of the engine's buffers on the device path)."""
    import torch

    dev = status.device
    hdr = torch.tensor([valid.numel(), status.numel(), hits.numel() // 16, payload.numel()], dtype=torch.int64,
                       device=dev).view(torch.uint8)
    return torch.cat([hdr, valid.view(torch.uint8), status.view(torch.uint8), hits.view(torch.uint8),
                      payload.view(torch.uint8)])


def wire_unpack(buf):
    """numpy views of a wire buffer: (valid i8, status i8, hits u32[n,4], payload u8)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8))
    n7, n8, nh, nb = (int(x) for x in b[:WIRE_HEADER].view(np.int64))
    o = WIRE_HEADER
    valid = b[o:o + n7].view(np.int8)
    o += n7
    status = b[o:o + n8].view(np.int8)
    o += n8
    hits = b[o:o + 16 * nh].view(np.uint32).reshape(nh, 4)
    o += 16 * nh
    payload = b[o:o + nb]
    if o + nb != len(b):
        raise ValueError(f"wire buffer of {len(b)} B, header says {o + nb} B")
    return valid, status, hits, payload


def decode_hits(status, hits):
    """Per-query (count, offset) from the hit list: SOME -> its payload
    offset, OVERFLOW / ABORTED -> the exact count (no payload); 0 elsewhere."""
    n = len(status)
    count = np.zeros(n, np.uint64)
    offset = np.zeros(n, np.uint64)
    if len(hits):
        q = hits[:, 0].astype(np.int64)
        word = hits[:, 2].astype(np.uint64) | (hits[:, 3].astype(np.uint64) << np.uint64(32))
        some = status[q] == SST_SOME
        count[q] = np.where(some, hits[:, 1].astype(np.uint64), word)
        offset[q] = np.where(some, word, 0)
    return count, offset


def candidates(payload, count, offset, i):
    """Row-index tuples of query i from a decoded result."""
    out, p = [], int(offset[i])
    for _ in range(int(count[i])):
        k = int(payload[p])
        out.append(tuple(int(x) for x in payload[p + 1:p + 1 + k]))
        p += 1 + k
    return out
