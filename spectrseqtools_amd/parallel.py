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

Wire format of one rank's result (wire_pack / wire_unpack, v3), packed on
the device with a few tensor ops (no host round trip): 2-bit is_valid and
status codes, 4 B per pair-path hit (its first pair-list entry and count:
the receiver rebuilds the candidates from its own copy of the table's pair
list, so those hits send no payload), 12-B records and the payload for the
few hits of the deferred paths.  About 0.35 B per query + 4 B per hit:
~10 MB per rank per config-3 step (v2, 12-B records + the dense payload:
33 MB; the engine's own layout: 51 MB).  wire_unpack + decode_hits +
candidates read it back with numpy alone.
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
WIRE_MAGIC = 0x3357545353  # "SSTW3"
SST_NONE, SST_EMPTY, SST_SOME, SST_OUT_OF_TABLE, SST_OVERFLOW, SST_ABORTED = 0, 1, 2, -1, -2, -4
SCAN_WAVES_PER_WG = 16  # k_explain_scan: 1024-lane workgroups


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


def pair_key(recs):
    """63-bit FNV-1a of a table's pair records (sst_table_pair_records): the
    receiver checks it decodes pair hits against the sender's pair list."""
    h = 0xCBF29CE484222325
    for b in np.ascontiguousarray(recs, dtype=np.uint32).tobytes():
        h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h & 0x7FFFFFFFFFFFFFFF


def scan_order_key(q, n, n_wg):
    """Sort key of queries q (int64) in the pair scan's hit order for a batch
    of n queries on n_wg workgroups: workgroup, its wave, the wave's tile
    round, lane (include/sst.h, sst_result_pair_hits; sst_kernels.hip
    k_explain_scan's tile order)."""
    q = np.asarray(q, dtype=np.int64)
    n_waves = SCAN_WAVES_PER_WG * n_wg
    rounds = max(1, -(-((n + 63) // 64) // n_waves))
    tile, lane = q >> 6, q & 63
    vw, r = tile % n_waves, tile // n_waves
    t = vw >> 1
    b, w = t % n_wg, ((t // n_wg) << 1) | (vw & 1)
    return ((b * SCAN_WAVES_PER_WG + w) * rounds + r) * 64 + lane


def wire_pack(valid, status, hits, payload, refs=None, n_pair=0, pair_bytes=0, n_wg=0, key=0):
    """One rank's result in the wire format (v3) as a flat uint8 tensor on
    the parts' device, built with tensor ops (no host round trip).
    valid / status: int8 tensors (is_valid results, explain statuses); hits:
    the engine's dense hit list as a uint8 tensor (16-B records,
    sst_result_hit_list); payload: the dense payload (uint8); refs, n_pair,
    pair_bytes, n_wg: the pair-path part (sst_result_pair_hits, refs as a
    uint8 tensor of 2 B per pair hit); key: pair_key of the table's pair
    records.

      header   8 x i64: magic, n_valid, n_explain, n_pair, n_explicit,
               payload bytes, n_wg, key
      valid    2-bit codes (is_valid + 1: 0 raise, 1 False, 2 True), 4 per byte
      status   2-bit codes: 0 NONE, 1 EMPTY, 2 pair hit, 3 OUT_OF_TABLE or an
               explicit hit
      pairs    per pair hit, in the scan's order (scan_order_key): u16 first
               pair-list entry | 0x8000 for OVERFLOW, u16 count.  The
               candidates are the entries first .. first + count - 1: no payload
      explicit 12-B records {u32 query | kind << 30, u32 a, u32 b} of the other
               hits (deferred paths): kind 0 SOME (a = candidates, b = payload
               offset), 1 OVERFLOW / 2 ABORTED (a, b = the exact count)
      payload  the explicit hits' payload ([k][row_0..row_{k-1}] per candidate)
    """
    import torch

    dev = status.device
    st = status.view(torch.int8)
    r = hits.view(torch.int32).view(-1, 4)
    nh = r.shape[0]
    if not 0 <= n_pair <= nh or pair_bytes > payload.numel():
        raise ValueError("wire format: pair part larger than the result")
    if payload.numel() - pair_bytes >= (1 << 32):
        raise ValueError("wire format: explicit payload offsets are 32-bit")
    mark = torch.zeros(st.numel(), dtype=torch.bool, device=dev)
    if n_pair:
        mark[r[:n_pair, 0].long()] = True
    code8 = torch.where(st == SST_NONE, 0, torch.where(st == SST_EMPTY, 1, torch.where(mark, 2, 3))).to(torch.uint8)
    code7 = (valid.view(torch.int8) + 1).to(torch.uint8)
    if n_pair:
        pairs = torch.stack([refs.view(torch.int16)[:n_pair], r[:n_pair, 1].to(torch.int16)], dim=1)
    else:
        pairs = torch.zeros((0, 2), dtype=torch.int16, device=dev)
    e = r[n_pair:]
    if e.shape[0]:
        kind = st[e[:, 0].long()]
        kind = torch.where(kind == SST_OVERFLOW, 1, torch.where(kind == SST_ABORTED, 2, 0)).to(torch.int32)
        some = kind == 0
        rec = torch.stack([e[:, 0] | (kind << 30), torch.where(some, e[:, 1], e[:, 2]),
                           torch.where(some, ((e[:, 2].long() & 0xFFFFFFFF) - int(pair_bytes)).to(torch.int32),
                                       e[:, 3])], dim=1)
    else:
        rec = torch.zeros((0, 3), dtype=torch.int32, device=dev)
    hdr = torch.tensor([WIRE_MAGIC, valid.numel(), st.numel(), n_pair, nh - n_pair, payload.numel() - pair_bytes,
                        n_wg, key], dtype=torch.int64, device=dev)
    return torch.cat([hdr.view(torch.uint8), _pack2(code7), _pack2(code8), pairs.contiguous().view(torch.uint8).view(-1),
                      rec.contiguous().view(torch.uint8).view(-1), payload.view(torch.uint8)[pair_bytes:]])


def wire_size(n_valid, n_explain, n_hits, payload_bytes, n_pair=0, pair_bytes=0):
    """Bytes of wire_pack's buffer for a result of these sizes."""
    return (WIRE_HEADER + (n_valid + 3) // 4 + (n_explain + 3) // 4 + 4 * n_pair + 12 * (n_hits - n_pair)
            + payload_bytes - pair_bytes)


def wire_unpack(buf, recs=None):
    """numpy form of a wire buffer: (valid i8, status i8, hits u32[n,4] in
    the engine's record layout {query, count, word lo, word hi}, payload u8).
    recs: the table's pair records (sst_table_pair_records), needed when the
    buffer holds pair hits.  The pair hits' candidates are rebuilt from the
    pair list (dense, in scan order, no pad bytes) ahead of the explicit
    payload: the same candidates per query as the sender's result, in
    another payload layout (canonical_digest compares the two)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8))
    magic, n7, n8, npair, nexp, nb, n_wg, key = (int(x) for x in b[:64].view(np.int64))
    if magic != WIRE_MAGIC:
        raise ValueError("not a wire buffer")
    o = WIRE_HEADER
    k7, k8 = (n7 + 3) // 4, (n8 + 3) // 4
    valid = _unpack2(b[o:o + k7], n7).astype(np.int8) - 1
    o += k7
    code = _unpack2(b[o:o + k8], n8)
    o += k8
    pairs = b[o:o + 4 * npair].view(np.uint16).reshape(npair, 2)
    o += 4 * npair
    rec = b[o:o + 12 * nexp].view(np.uint32).reshape(nexp, 3)
    o += 12 * nexp
    xpay = b[o:o + nb]
    if o + nb != len(b):
        raise ValueError(f"wire buffer of {len(b)} B, header says {o + nb} B")
    status = np.select([code == 0, code == 1, code == 2], [SST_NONE, SST_EMPTY, SST_SOME], SST_OUT_OF_TABLE)
    status = status.astype(np.int8)
    # pair hits: the queries with code 2, in the scan's order
    qp = np.flatnonzero(code == 2)
    if len(qp) != npair:
        raise ValueError(f"wire buffer: {len(qp)} pair-hit codes, header says {npair}")
    ppay = np.zeros(0, np.uint8)
    phits = np.zeros((npair, 4), np.uint32)
    if npair:
        if recs is None or pair_key(recs) != key:
            raise ValueError("wire buffer: pair hits need the sender's pair records")
        recs = np.asarray(recs, dtype=np.uint32)
        qp = qp[np.argsort(scan_order_key(qp, n8, n_wg), kind="stable")]
        first = (pairs[:, 0] & 0x7FFF).astype(np.int64)
        ovf = (pairs[:, 0] >> 15).astype(bool)
        cnt = pairs[:, 1].astype(np.int64)
        status[qp] = np.where(ovf, SST_OVERFLOW, SST_SOME)
        c_some = np.where(ovf, 0, cnt)  # OVERFLOW: the count only
        starts = np.cumsum(c_some) - c_some
        idx = np.repeat(first - starts, c_some) + np.arange(int(c_some.sum()))
        r32 = recs[idx]
        lens = 1 + (r32 & 0xFF).astype(np.int64)
        ppay = r32.view(np.uint8).reshape(-1, 4)[np.arange(4)[None, :] < lens[:, None]]
        hb = np.zeros(npair, np.int64)  # payload bytes per hit
        if len(idx):
            owner = np.repeat(np.arange(npair), c_some)
            np.add.at(hb, owner, lens)
        off = np.cumsum(hb) - hb
        phits[:, 0] = qp
        phits[:, 1] = cnt
        phits[:, 2] = np.where(ovf, cnt, off & 0xFFFFFFFF)
        phits[:, 3] = np.where(ovf, 0, off >> 32)
    q = (rec[:, 0] & 0x3FFFFFFF).astype(np.int64)
    kind = rec[:, 0] >> 30
    status[q] = np.select([kind == 1, kind == 2], [SST_OVERFLOW, SST_ABORTED], SST_SOME)
    ehits = np.zeros((nexp, 4), np.uint32)
    ehits[:, 0] = q
    some = kind == 0
    xoff = rec[:, 2].astype(np.uint64) + np.uint64(len(ppay))
    ehits[:, 1] = np.where(some, rec[:, 1], np.minimum(rec[:, 1].astype(np.uint64) | (rec[:, 2].astype(np.uint64) << 32),
                                                          0xFFFFFFFF)).astype(np.uint32)
    ehits[:, 2] = np.where(some, xoff & np.uint64(0xFFFFFFFF), rec[:, 1])
    ehits[:, 3] = np.where(some, xoff >> np.uint64(32), rec[:, 2])
    return valid, status, np.concatenate([phits, ehits]), np.concatenate([ppay, xpay])


def canonical_digest(status, count, offset, payload):
    """SHA-256 of a result independent of its payload layout: status bytes,
    per-query counts, and the candidate bytes of every SOME query in query
    order (offsets and pad bytes are layout, not result)."""
    import hashlib

    status = np.asarray(status, dtype=np.int8)
    count = np.asarray(count, dtype=np.uint64)
    payload = np.asarray(payload, dtype=np.uint8)
    qs = np.flatnonzero(status == SST_SOME)
    beg = np.asarray(offset, dtype=np.int64)[qs]
    c = count[qs].astype(np.int64)
    pos = beg.copy()
    act = np.flatnonzero(c > 0)
    step = 0
    while len(act):
        pos[act] += 1 + payload[pos[act]].astype(np.int64)
        step += 1
        act = act[c[act] > step]
    ln = pos - beg
    idx = np.repeat(beg - (np.cumsum(ln) - ln), ln) + np.arange(int(ln.sum()))
    h = hashlib.sha256()
    for a in (status, count, ln, payload[idx]):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


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
