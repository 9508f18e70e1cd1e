"""One rank of the world-size-2 gloo test (tests/test_parallel.py): the
multi-GPU layer's host logic on CPU -- sharding, the agreed-size gather of
per-rank result buffers to rank 0, and the max-over-ranks step time that
bench.py reports."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from spectrseqtools_amd.parallel import Gatherer, dist_env, shard_by_weight, shard_range  # noqa: E402


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
