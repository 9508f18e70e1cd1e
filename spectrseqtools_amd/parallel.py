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

Wire format of one rank's result (v5, include/sst.h sst_wire_pack): packed
on the device by one kernel (no host round trip): 1-bit is_valid codes,
1-bit hit flags per explain query (SOME / OVERFLOW / ABORTED; EMPTY and the
other rare statuses in the list), per pair-path hit its
first pair-list entry in w = ceil(log2(pair-list entries)) bits and a 3-bit
count code ( the receiver rebuilds the candidates from its own copy of the
table's pair list, so those hits send no payload), 12-B records and the
payload for the few hits of the deferred paths, and a list of the rare rest
(is_valid raises, statuses other than NONE / SOME, counts outside 1..7).
About 0.125 B per is_valid query, 0.125 B per explain query and ~2 B per
pair hit: ~5.4 MB per rank per config-3 step (v4, 2-bit status codes: 6.7
MB; v3, 2-bit codes and 4 B per pair hit: 10.7 MB; v2, 12-B records + the
dense payload: 33 MB; the engine's own layout: 51 MB).
wire_pack_host states the packer in numpy; wire_unpack + decode_hits +
candidates read a buffer back with numpy alone.
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

    def agree(self, nbytes, capacity=None):
        """All-gather every rank's byte count (one int64 each); rank 0 keeps
        receive buffers of `capacity` bytes (default: the agreed maximum) and
        reuses them while later agreements fit (a per-step agreement costs the
        one small all_gather, no allocation)."""
        import torch

        t = torch.tensor([int(nbytes)], dtype=torch.int64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(out, t)
        self.sizes = [int(x.item()) for x in out]
        self.max = max(self.sizes) if self.sizes else 0
        if self.dist.get_rank() == 0:
            cap = max(self.max, int(capacity or 0))
            if self.recv is None or self.recv[0].numel() < self.max:
                self.recv = [torch.empty(cap, dtype=torch.uint8, device=self.device)
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
        elif buf.numel() > self.max:  # a buffer with room past its used bytes: send the agreed size only
            buf = buf[:self.max]
        if rank == 0:
            self.dist.gather(buf, gather_list=[r[:self.max] for r in self.recv], dst=0)
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


WIRE_HEADER = 128
WIRE_MAGIC = 0x3557545353  # "SSTW5"
SST_NONE, SST_EMPTY, SST_SOME, SST_OUT_OF_TABLE, SST_OVERFLOW, SST_ABORTED = 0, 1, 2, -1, -2, -4
SCAN_WAVES_PER_WG = 16  # k_explain_scan: 1024-lane workgroups
LIST_RAISE, LIST_STATUS, LIST_COUNT = 0, 1, 2  # wire list entry types


def _pack3(codes):
    """codes in {0..7} -> 10 per little-endian u32 (bits 3k..3k+2), as bytes."""
    c = np.asarray(codes, dtype=np.uint32)
    c = np.concatenate([c, np.zeros((-len(c)) % 10, np.uint32)]).reshape(-1, 10)
    return (c << (3 * np.arange(10, dtype=np.uint32))).sum(axis=1, dtype=np.uint32).view(np.uint8)


def _unpack3(b, n):
    w = np.asarray(b, dtype=np.uint8)[:4 * ((n + 9) // 10)].view(np.uint32)
    return ((w[:, None] >> (3 * np.arange(10, dtype=np.uint32))) & 7).ravel()[:n].astype(np.int64)


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
    k_explain_scan's tile order); n_wg = 0: query order (the rows step)."""
    q = np.asarray(q, dtype=np.int64)
    if n_wg == 0:  # a rows-step result (sst_step_rows_device): its hits come in query order
        return q
    n_waves = SCAN_WAVES_PER_WG * n_wg
    rounds = max(1, -(-((n + 63) // 64) // n_waves))
    tile, lane = q >> 6, q & 63
    vw, r = tile % n_waves, tile // n_waves
    t = vw >> 1
    b, w = t % n_wg, ((t // n_wg) << 1) | (vw & 1)
    return ((b * SCAN_WAVES_PER_WG + w) * rounds + r) * 64 + lane


def _a8(x):
    return (int(x) + 7) & ~7


def first_width(n_entries):
    """Bits per pair hit's first entry: ceil(log2(pair-list entries)), >= 1."""
    w = 1
    while (1 << w) < n_entries:
        w += 1
    return w


def wire_layout(n_valid, n_explain, n_pair, n_explicit, xpay, w):
    """Byte offsets of the wire v5 sections (include/sst.h, sst_wire_pack):
    every section starts 8-byte aligned; 'list' is the fixed part's size."""
    o = {"valid": WIRE_HEADER}
    o["status"] = o["valid"] + _a8((n_valid + 7) // 8)
    o["first"] = o["status"] + _a8((n_explain + 7) // 8)
    o["codes"] = o["first"] + 8 * ((n_pair * w + 63) // 64)
    o["explicit"] = o["codes"] + 8 * ((n_pair + 19) // 20)
    o["payload"] = o["explicit"] + _a8(12 * n_explicit)
    o["list"] = o["payload"] + _a8(xpay)
    return o


def wire_pack_host(valid, status, hits, payload, refs=None, n_pair=0, pair_bytes=0, n_wg=0, recs=None):
    """numpy statement of sst_wire_pack (the device packer of the gather's
    wire format v5) for host-side results: valid / status int8 arrays, hits
    the dense hit list as u32 [n, 4] {query, count, word lo, word hi}, payload
    u8, refs u16 per pair hit (first | 0x8000 for OVERFLOW), recs the table's
    pair records.  Same bytes as the device packer except the list entries'
    order (here: by type, then index)."""
    valid = np.asarray(valid, dtype=np.int8)
    st = np.asarray(status, dtype=np.int8)
    hits = np.asarray(hits, dtype=np.uint32).reshape(-1, 4)
    payload = np.asarray(payload, dtype=np.uint8)
    nh, n7, n8 = len(hits), len(valid), len(st)
    if not 0 <= n_pair <= nh or pair_bytes > len(payload):
        raise ValueError("wire format: pair part larger than the result")
    if n7 >= 1 << 30 or n8 >= 1 << 30:
        raise ValueError("wire format: list entries index at most 2^30 queries")
    n_exp, xpay = nh - n_pair, len(payload) - pair_bytes
    if xpay >= 1 << 32:
        raise ValueError("wire format: explicit payload offsets are 32-bit")
    E = len(recs) if (n_pair and recs is not None) else 0
    w = first_width(E)
    o = wire_layout(n7, n8, n_pair, n_exp, xpay, w)
    # list entries
    lst = []
    for q in np.flatnonzero(valid == -1):
        lst.append((LIST_RAISE, int(q), 0))
    for q in np.flatnonzero((st != SST_NONE) & (st != SST_SOME)):
        lst.append((LIST_STATUS, int(q), int(np.uint8(st[q]))))
    cnt = hits[:n_pair, 1].astype(np.int64)
    for i in np.flatnonzero((cnt < 1) | (cnt > 7)):
        lst.append((LIST_COUNT, int(i), int(cnt[i])))
    buf = np.zeros(o["list"] + 8 * len(lst), np.uint8)
    hdr = [WIRE_MAGIC, n7, n8, n_pair, n_exp, xpay, n_wg, pair_key(recs) if n_pair else 0, w, len(lst), len(lst),
           o["list"], 0, 0, 0, 0]
    buf[:WIRE_HEADER] = np.array(hdr, dtype=np.uint64).view(np.uint8)
    vb = np.packbits(valid == 1, bitorder="little")
    buf[o["valid"]:o["valid"] + len(vb)] = vb
    hit = (st == SST_SOME) | (st == SST_OVERFLOW) | (st == SST_ABORTED)
    sb = np.packbits(hit, bitorder="little")
    buf[o["status"]:o["status"] + len(sb)] = sb
    if n_pair:
        f = np.asarray(refs, dtype=np.uint16)[:n_pair].astype(np.int64) & 0x7FFF
        fb = np.packbits(((f[:, None] >> np.arange(w)) & 1).astype(np.uint8).ravel(), bitorder="little")
        buf[o["first"]:o["first"] + len(fb)] = fb
        cb = _pack3(np.where((cnt >= 1) & (cnt <= 7), cnt, 0))
        buf[o["codes"]:o["codes"] + len(cb)] = cb
    e = hits[n_pair:]
    if n_exp:
        s = st[e[:, 0].astype(np.int64)]
        kind = np.where(s == SST_OVERFLOW, 1, np.where(s == SST_ABORTED, 2, 0)).astype(np.uint32)
        some = kind == 0
        off = ((e[:, 2].astype(np.uint64) | (e[:, 3].astype(np.uint64) << np.uint64(32))) - np.uint64(pair_bytes))
        rec = np.stack([e[:, 0] | (kind << np.uint32(30)), np.where(some, e[:, 1], e[:, 2]),
                        np.where(some, (off & np.uint64(0xFFFFFFFF)).astype(np.uint32), e[:, 3])], axis=1)
        buf[o["explicit"]:o["explicit"] + 12 * n_exp] = rec.astype(np.uint32).view(np.uint8).ravel()
    buf[o["payload"]:o["payload"] + xpay] = payload[pair_bytes:]
    if lst:
        ent = np.array([((t << 30) | i, v) for t, i, v in lst], dtype=np.uint32)
        buf[o["list"]:] = ent.view(np.uint8).ravel()
    return buf


def wire_unpack(buf, recs=None):
    """numpy form of a wire v5 buffer (sst_wire_pack / wire_pack_host; a
    gathered buffer may carry padding after its list): (valid i8, status i8,
    hits u32[n,4] in the engine's record layout {query, count, word lo, word
    hi}, payload u8).  recs: the table's pair records
    (sst_table_pair_records), needed when the buffer holds pair hits.  The
    pair hits' candidates are rebuilt from the pair list (dense, in scan
    order, no pad bytes) ahead of the explicit payload: the same candidates
    per query as the sender's result, in another payload layout
    (canonical_digest compares the two)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8))
    if len(b) < WIRE_HEADER:
        raise ValueError("not a wire buffer")
    h = [int(x) for x in b[:WIRE_HEADER].view(np.uint64)]
    magic, n7, n8, npair, nexp, nb, n_wg, key, w, n_list, list_cap, o_list = h[:12]
    if magic != WIRE_MAGIC:
        raise ValueError("not a wire buffer")
    o = wire_layout(n7, n8, npair, nexp, nb, w)
    if o["list"] != o_list:
        raise ValueError("wire buffer: header and layout disagree")
    if n_list > list_cap or o_list + 8 * n_list > len(b):
        raise ValueError(f"wire buffer: {n_list} list entries, room for {min(list_cap, (len(b) - o_list) // 8)}")
    ent = b[o_list:o_list + 8 * n_list].view(np.uint32).reshape(n_list, 2)
    typ, idx, val = ent[:, 0] >> 30, (ent[:, 0] & 0x3FFFFFFF).astype(np.int64), ent[:, 1]
    valid = np.unpackbits(b[o["valid"]:o["status"]], bitorder="little")[:n7].astype(np.int8)
    valid[idx[typ == LIST_RAISE]] = -1
    hit = np.unpackbits(b[o["status"]:o["first"]], bitorder="little")[:n8].astype(bool)
    status = np.where(hit, SST_SOME, SST_NONE).astype(np.int8)
    m = typ == LIST_STATUS
    status[idx[m]] = val[m].astype(np.uint8).view(np.int8)
    rec = b[o["explicit"]:o["explicit"] + 12 * nexp].view(np.uint32).reshape(nexp, 3)
    q = (rec[:, 0] & 0x3FFFFFFF).astype(np.int64)
    kind = rec[:, 0] >> 30
    # pair hits: the hit bits of queries without an explicit record, in the scan's order
    pmask = hit.copy()
    pmask[q] = False
    qp = np.flatnonzero(pmask)
    if len(qp) != npair:
        raise ValueError(f"wire buffer: {len(qp)} pair hits flagged, header says {npair}")
    ppay = np.zeros(0, np.uint8)
    phits = np.zeros((npair, 4), np.uint32)
    if npair:
        if recs is None or pair_key(recs) != key:
            raise ValueError("wire buffer: pair hits need the sender's pair records")
        recs = np.asarray(recs, dtype=np.uint32)
        qp = qp[np.argsort(scan_order_key(qp, n8, n_wg), kind="stable")]
        fb = np.unpackbits(b[o["first"]:o["codes"]], bitorder="little")[:npair * w].reshape(npair, w)
        first = fb.astype(np.int64) @ (np.int64(1) << np.arange(w, dtype=np.int64))
        cnt = _unpack3(b[o["codes"]:o["explicit"]], npair)
        m = typ == LIST_COUNT
        cnt[idx[m]] = val[m]
        ovf = status[qp] == SST_OVERFLOW
        status[qp] = np.where(ovf, SST_OVERFLOW, SST_SOME)
        c_some = np.where(ovf, 0, cnt)  # OVERFLOW: the count only
        starts = np.cumsum(c_some) - c_some
        ix = np.repeat(first - starts, c_some) + np.arange(int(c_some.sum()))
        r32 = recs[ix]
        lens = 1 + (r32 & 0xFF).astype(np.int64)
        ppay = r32.view(np.uint8).reshape(-1, 4)[np.arange(4)[None, :] < lens[:, None]]
        hb = np.zeros(npair, np.int64)  # payload bytes per hit
        if len(ix):
            np.add.at(hb, np.repeat(np.arange(npair), c_some), lens)
        off = np.cumsum(hb) - hb
        phits[:, 0] = qp
        phits[:, 1] = cnt
        phits[:, 2] = np.where(ovf, cnt, off & 0xFFFFFFFF)
        phits[:, 3] = np.where(ovf, 0, off >> 32)
    xpay = b[o["payload"]:o["payload"] + nb]
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


def wire_used_bytes(buf):
    """Bytes a packed wire buffer uses: its fixed part plus its list."""
    h = np.asarray(buf[:WIRE_HEADER], dtype=np.uint8).view(np.uint64)
    return int(h[11]) + 8 * int(h[9])


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
