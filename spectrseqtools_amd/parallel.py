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

Wire format of one rank's result (wire_pack / wire_unpack), packed on the
device with a few tensor ops (no host round trip):
  header   8 x i64: magic, n_valid, n_explain, n_hits, payload_bytes, 0, 0, 0
  valid    2-bit codes (is_valid + 1: 0 raise, 1 False, 2 True), 4 per byte
  status   2-bit codes: 0 NONE, 1 EMPTY, 2 a hit record follows, 3 OUT_OF_TABLE
  hits     12-B records {u32 query | kind << 30, u32 a, u32 b}: kind 0 SOME
           (a = candidates, b = their payload offset), 1 OVERFLOW / 2 ABORTED
           (a, b = the exact count's low / high word, no payload)
  payload  the dense payload ([k][row_0..row_{k-1}] per candidate)
About 0.5 B per query + 12 B per query with candidates + payload: 33 MB per
rank per config-3 step instead of the 51 MB of the engine's own layout
(1 B status, 16-B hit records).  wire_unpack + decode_hits + candidates read
it back with numpy alone.
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


WIRE_HEADER = 64
WIRE_MAGIC = 0x3257545353  # "SSTW2"
SST_NONE, SST_EMPTY, SST_SOME, SST_OUT_OF_TABLE, SST_OVERFLOW, SST_ABORTED = 0, 1, 2, -1, -2, -4


def _pack2(codes):
    """uint8 codes in {0..3} -> 4 per byte (torch, on the codes' device)."""
    import torch

    n = codes.numel()
    pad = (-n) % 4
    if pad:
        codes = torch.cat([codes, torch.zeros(pad, dtype=torch.uint8, device=codes.device)])
    c = codes.view(-1, 4)
    return c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)


def _unpack2(b, n):
    b = np.asarray(b, dtype=np.uint8)
    c = np.stack([b & 3, (b >> 2) & 3, (b >> 4) & 3, b >> 6], axis=1).ravel()
    return c[:n]


def wire_pack(valid, status, hits, payload):
    """One rank's result in the wire format above, as a flat uint8 tensor on
    the parts' device.  valid / status: int8 tensors (is_valid results,
    explain statuses); hits: the engine's dense hit list as a uint8 tensor
    (16-B records, include/sst.h sst_result_hit_list); payload: uint8."""
    import torch

    dev = status.device
    st = status.view(torch.int8)
    code8 = torch.where(st == SST_NONE, 0, torch.where(st == SST_EMPTY, 1, torch.where(st == SST_OUT_OF_TABLE, 3, 2)))
    code7 = (valid.view(torch.int8) + 1).to(torch.uint8)
    r = hits.view(torch.int32).view(-1, 4)
    if payload.numel() >= (1 << 32):
        raise ValueError("wire format: payload offsets are 32-bit")
    if r.shape[0]:
        kind = st[r[:, 0].long()]
        kind = torch.where(kind == SST_OVERFLOW, 1, torch.where(kind == SST_ABORTED, 2, 0)).to(torch.int32)
        some = kind == 0
        rec = torch.stack([r[:, 0] | (kind << 30), torch.where(some, r[:, 1], r[:, 2]),
                           torch.where(some, r[:, 2], r[:, 3])], dim=1)
    else:
        rec = torch.zeros((0, 3), dtype=torch.int32, device=dev)
    hdr = torch.tensor([WIRE_MAGIC, valid.numel(), status.numel(), r.shape[0], payload.numel(), 0, 0, 0],
                       dtype=torch.int64, device=dev)
    return torch.cat([hdr.view(torch.uint8), _pack2(code7), _pack2(code8.to(torch.uint8)),
                      rec.contiguous().view(torch.uint8).view(-1), payload.view(torch.uint8)])


def wire_unpack(buf):
    """numpy form of a wire buffer: (valid i8, status i8, hits u32[n,4] in
    the engine's record layout {query, count, word lo, word hi}, payload u8)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8))
    magic, n7, n8, nh, nb = (int(x) for x in b[:40].view(np.int64))
    if magic != WIRE_MAGIC:
        raise ValueError("not a wire buffer")
    o = WIRE_HEADER
    k7, k8 = (n7 + 3) // 4, (n8 + 3) // 4
    valid = _unpack2(b[o:o + k7], n7).astype(np.int8) - 1
    o += k7
    code = _unpack2(b[o:o + k8], n8)
    o += k8
    rec = b[o:o + 12 * nh].view(np.uint32).reshape(nh, 3)
    o += 12 * nh
    payload = b[o:o + nb]
    if o + nb != len(b):
        raise ValueError(f"wire buffer of {len(b)} B, header says {o + nb} B")
    status = np.select([code == 0, code == 1, code == 3], [SST_NONE, SST_EMPTY, SST_OUT_OF_TABLE], SST_SOME)
    status = status.astype(np.int8)
    q = (rec[:, 0] & 0x3FFFFFFF).astype(np.int64)
    kind = rec[:, 0] >> 30
    status[q] = np.select([kind == 1, kind == 2], [SST_OVERFLOW, SST_ABORTED], SST_SOME)
    hits = np.zeros((nh, 4), np.uint32)
    hits[:, 0] = q
    some = kind == 0
    hits[:, 1] = np.where(some, rec[:, 1], np.minimum(rec[:, 1].astype(np.uint64) | (rec[:, 2].astype(np.uint64) << 32),
                                                         0xFFFFFFFF)).astype(np.uint32)
    hits[:, 2] = np.where(some, rec[:, 2], rec[:, 1])
    hits[:, 3] = np.where(some, 0, rec[:, 2])
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
