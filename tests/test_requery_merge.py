"""The skeleton walk's merged re-query answers (sst_requery_merge_device via
pipeline_device.merge_requery_round): over several rounds every side reads
its k-th answer at start + k, in the order the rounds produced them -- what
k_skel_walk's resolved() expects of a single merged round."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_merged_rounds_are_per_side_round_major():
    import torch

    from spectrseqtools_amd import _native
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.pipeline_device import merge_requery_round

    eng = _native.get_engine(0)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=SequenceInformation(6, 1000.0, 1000.0, 0.5), engine=eng)
    dev = torch.device("cuda", eng.device)
    rng = np.random.default_rng(3)
    n_sides = 3037  # more sides than one scan chunk's threads
    want = {sd: [] for sd in range(n_sides)}
    merged, n_merged = None, 0
    tag = 0
    for rnd in range(6):
        # a round: some sides request a contiguous block each, blocks in arbitrary order
        sides = rng.choice(n_sides, size=int(rng.integers(1, 900)), replace=False)
        counts = rng.integers(1, 5, len(sides))
        perm = rng.permutation(len(sides))
        block = np.zeros(n_sides, np.int64)
        total = int(counts.sum())
        p_ = np.zeros(total, np.int64)
        pos = 0
        for j in perm:  # the lanes' atomicAdd order
            sd, c = int(sides[j]), int(counts[j])
            block[sd] = (pos << 32) | c
            for k in range(c):
                tag += 1
                p_[pos + k] = tag
                want[sd].append(tag)
            pos += c
        t = lambda x: torch.as_tensor(x, device=dev)  # noqa: E731
        merged, n_merged = merge_requery_round(dp, merged, n_merged, t(block), t(p_), t((p_ % 7).astype(np.int32)),
                                               t((p_ % 3).astype(np.int8)), n_sides)
        eng.synchronize()
        blk, ptr, nn, st = (x.cpu().numpy() for x in merged)
        assert n_merged == sum(len(v) for v in want.values())
        for sd in range(n_sides):
            start, cnt = int(blk[sd]) >> 32, int(blk[sd]) & 0xFFFFFFFF
            got = ptr[start:start + cnt].tolist()
            assert got == want[sd], (rnd, sd)
            assert nn[start:start + cnt].tolist() == [x % 7 for x in want[sd]]
            assert st[start:start + cnt].tolist() == [x % 3 for x in want[sd]]
    dp.close()
