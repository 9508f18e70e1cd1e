"""One rank of the world-size-2 gloo test (tests/test_parallel.py): the
multi-GPU layer's host logic on CPU -- sharding, the agreed-size gather of
per-rank result buffers to rank 0, the engine's result wire format (each
rank encodes oracle answers to its own queries exactly as the engine lays out
a result: status bytes, dense hit list -- the pair-path hits first, in the
scan's order, with their pair-list refs --, dense payload; rank 0 decodes
every query of every rank from the wire and its copy of the pair list and
checks it), and the max-over-ranks step time that bench.py reports."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), HERE]
import _oracle as oracle  # noqa: E402  (test infrastructure: the answers each rank encodes)
from spectrseqtools_amd.parallel import (Gatherer, candidates, decode_hits, dist_env, pair_key,  # noqa: E402
                                         scan_order_key, shard_by_weight, shard_range, wire_pack_host, wire_unpack)

ROWS = [0, 305042, 306026, 329053, 345048]  # canonical alphabet (a 5 x 377 397 table)
TOL, PREC, CAP = 1e-5, 1e-3, 1


def rank_queries(rank, n=600):
    rng = np.random.default_rng(1000 + rank)
    k = rng.integers(1, 5, n)
    m = np.array([sum(ROWS[1:][j] for j in rng.integers(0, 4, kk)) for kk in k]) * PREC
    m = m + rng.normal(0, 0.003, n)
    m[:20] = rng.uniform(0.0, 0.2, 20)  # below the first reachable mass: NONE / EMPTY
    t = TOL * rng.uniform(300, 3000, n)
    t[20:120] = rng.uniform(1.0, 3.0, 100)  # wide windows: several candidates (OVERFLOW past CAP)
    m[120:130], t[120:130] = rng.uniform(648.0, 652.0, 10), 45.0  # all 10 two-row sums: listed counts (> 7)
    m[130:135] = 1e5  # beyond the table: is_valid raises, explain OUT_OF_TABLE
    return m, t


def oracle_answers(table, alph, masses, thr):
    out = []
    for m, t in zip(masses, thr):
        st, sols, n_empty, _ = oracle.explain_table(table, 32, alph, float(m), float(t), TOL, -1)
        out.append((st, sorted(sols), n_empty))
    return out


def pair_list(rows):
    """The scan's pair list for these row masses (sst_api.cpp build_pair_list):
    every single row and every two-row sum below 3 * w_min, by (sum, top
    row); (sums, payload records [k][rows] as u32)."""
    w_min, e = min(rows[1:]), []
    for r1 in range(1, len(rows)):
        e.append((rows[r1], r1, 1 | (r1 << 8)))
        for r2 in range(1, r1 + 1):
            if rows[r1] + rows[r2] < 3 * w_min:
                e.append((rows[r1] + rows[r2], r1, 2 | (r2 << 8) | (r1 << 16)))
    e.sort(key=lambda x: (x[0], x[1]))
    return np.array([x[0] for x in e], np.int64), np.array([x[2] for x in e], np.uint32)


def rec_bytes(rec):
    k = int(rec) & 0xFF
    return [k] + [(int(rec) >> (8 * (j + 1))) & 0xFF for j in range(k)]


def engine_layout(answers, masses, thr, sums, recs, n_wg):
    """An engine result (include/sst.h) built from oracle answers, as a fused
    device pass lays it out: status bytes; the dense hit list -- first the
    pair-path hits (windows below 3 * w_min whose candidates are the pair-list
    entries with sums in the window), in the scan's order, with their refs
    (first entry | 0x8000 for OVERFLOW, sst_result_pair_hits), then the other
    hits --; the dense payload (pair-path candidates + 2 pad bytes per query,
    then the others').  Returns (status, hits, payload, refs, n_pair, pair_bytes)."""
    n = len(answers)
    w_min = min(ROWS[1:])
    status = np.zeros(n, np.int8)
    pair, other = [], []
    for i, (st, sols, n_empty) in enumerate(answers):
        if st == 1 and sols:
            over = len(sols) > CAP
            status[i] = -2 if over else 2  # SST_OVERFLOW: exact count, no payload
            lo = int(np.rint(masses[i] / PREC)) - int(np.ceil(thr[i] / PREC))
            hi = int(np.rint(masses[i] / PREC)) + int(np.ceil(thr[i] / PREC))
            a, b = np.searchsorted(sums, max(lo, 1), "left"), np.searchsorted(sums, hi, "right")
            ents = sorted(tuple(rec_bytes(r)[1:]) for r in recs[a:b])
            if hi < 3 * w_min and ents == sorted(tuple(c) for c in sols):
                pair.append((i, int(a), int(b - a), over))
            else:
                other.append((i, sols, over))
        elif st == -1:
            status[i] = -1  # SST_OUT_OF_TABLE
        else:
            status[i] = 1 if (st == 1 and n_empty) else 0
    pair.sort(key=lambda x: int(scan_order_key([x[0]], n, n_wg)[0]))
    hits, refs, payload = [], [], []
    for i, first, cnt, over in pair:
        refs.append(first | (0x8000 if over else 0))
        if over:
            hits.append([i, cnt, cnt, 0])
        else:
            hits.append([i, cnt, len(payload), 0])
            for r in recs[first:first + cnt]:
                payload += rec_bytes(r)
            payload += [0, 0]  # the scan's 2 pad bytes after a query's candidates
    pair_bytes = len(payload)
    for i, sols, over in other:
        if over:
            hits.append([i, len(sols), len(sols), 0])
        else:
            hits.append([i, len(sols), len(payload), 0])
            for c in sols:
                payload += [len(c)] + list(c)
    return (status, np.array(hits, np.uint32).reshape(-1, 4), np.array(payload, np.uint8),
            np.array(refs, np.uint16), len(pair), pair_bytes)


def main():
    rank, world, _local = dist_env()
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world == 2

    # contiguous balanced shards covering every item exactly once
    for n in (0, 1, 7, 10_000, 10_001):
        mine = torch.tensor(shard_range(n, rank, world), dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, mine)
        bounds = [tuple(int(x) for x in t) for t in allr]
        assert bounds[0][0] == 0 and bounds[-1][1] == n
        assert all(bounds[k][1] == bounds[k + 1][0] for k in range(world - 1))
        sizes = [b - a for a, b in bounds]
        assert max(sizes) - min(sizes) <= 1

    # weight-balanced shards (spectra by query count) agree on every rank
    w = np.random.default_rng(5).integers(1, 400, 1000)
    cuts = shard_by_weight(w, world)
    assert cuts[0][0] == 0 and cuts[-1][1] == len(w) and cuts[0][1] == cuts[1][0]
    loads = [w[a:b].sum() for a, b in cuts]
    assert abs(loads[0] - loads[1]) <= w.max()

    # per-rank result buffers of different sizes -> rank 0, byte-exact
    rng = np.random.default_rng(100 + rank)
    mine = torch.from_numpy(rng.integers(0, 256, 1000 + 37 * rank, dtype=np.uint8))
    g = Gatherer(dist, torch.device("cpu"))
    sizes = g.agree(mine.numel())
    assert sizes == [1000, 1037]
    got = g.gather(mine)
    if rank == 0:
        for r, buf in enumerate(got):
            want = np.random.default_rng(100 + r).integers(0, 256, 1000 + 37 * r, dtype=np.uint8)
            assert np.array_equal(buf.numpy(), want), r
    else:
        assert got is None

    # the engine's wire format: every rank's answers decode on rank 0
    table = oracle.build_table(ROWS, max(ROWS) * 35, 32)
    alph = oracle.Alphabet(ROWS, [0] * 5, [20] * 5)
    masses, thr = rank_queries(rank)
    ans = oracle_answers(table, alph, masses, thr)
    sums, recs = pair_list(ROWS)
    n_wg = 1 + rank  # the scan grid differs per rank: each buffer carries its own
    st, hits, pay, refs, n_pair, pair_bytes = engine_layout(ans, masses, thr, sums, recs, n_wg)
    assert 0 < n_pair < len(hits)  # both kinds of hit records travel
    valid = np.array([oracle.is_valid(table, 32, m, t, TOL) for m, t in zip(masses, thr)], np.int8)
    wire = wire_pack_host(valid, st, hits, pay, refs, n_pair, pair_bytes, n_wg, recs)
    ent = wire[int(wire[88:96].view(np.uint64)[0]):].view(np.uint32).reshape(-1, 2)
    kinds = set((ent[:, 0] >> 30).tolist())
    assert kinds == {0, 1, 2}, kinds  # raises, statuses other than NONE / SOME, pair counts outside 1..7
    wire = torch.from_numpy(wire)
    g2 = Gatherer(dist, torch.device("cpu"))
    g2.agree(wire.numel())
    got = g2.gather(wire)
    if rank == 0:
        n_checked = n_some = n_over = 0
        for r, buf in enumerate(got):
            v_r, st_r, hits_r, pay_r = wire_unpack(buf.numpy(), recs)
            m_r, t_r = rank_queries(r)
            want = oracle_answers(table, alph, m_r, t_r)
            assert np.array_equal(v_r, [oracle.is_valid(table, 32, m, t, TOL) for m, t in zip(m_r, t_r)])
            cnt, off = decode_hits(st_r, hits_r)
            for i, (s0, sols, n_empty) in enumerate(want):
                if s0 == 1 and len(sols) > CAP:
                    assert st_r[i] == -2 and int(cnt[i]) == len(sols), (r, i)
                    n_over += 1
                elif s0 == 1 and sols:
                    assert st_r[i] == 2 and sorted(candidates(pay_r, cnt, off, i)) == sols, (r, i)
                    n_some += 1
                elif s0 == -1:
                    assert st_r[i] == -1, (r, i)
                else:
                    assert st_r[i] == (1 if (s0 == 1 and n_empty) else 0), (r, i)
                n_checked += 1
        assert n_checked == 1200 and n_some > 0 and n_over > 0, (n_checked, n_some, n_over)
    else:
        assert got is None

    # bench.py: step time = max over ranks; value = all ranks' peaks / that time
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    pk = torch.tensor([100 * (rank + 1)], dtype=torch.int64)
    dist.all_reduce(pk)
    assert float(t.item()) == 1.5 and int(pk.item()) == 300

    dist.barrier()
    dist.destroy_process_group()
    print(f"ok rank {rank}", flush=True)


if __name__ == "__main__":
    main()
