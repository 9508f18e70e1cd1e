"""The skeleton walk's merged re-query answers (pipeline_device.
merge_requery_round, host logic on CPU tensors): over several rounds every
side reads its k-th answer at start + k, in the order the rounds produced
them -- what k_skel_walk's resolved() expects of a single merged round."""
import numpy as np
import torch

from spectrseqtools_amd.pipeline_device import merge_requery_round


def test_merged_rounds_are_per_side_round_major():
    rng = np.random.default_rng(3)
    n_sides = 37
    want = {sd: [] for sd in range(n_sides)}
    m_sid = torch.zeros(0, dtype=torch.int64)
    m_ptr = torch.zeros(0, dtype=torch.int64)
    m_n = torch.zeros(0, dtype=torch.int32)
    m_st = torch.zeros(0, dtype=torch.int8)
    tag = 0
    for rnd in range(6):
        # a round: some sides request a contiguous block each, blocks in arbitrary order
        sides = rng.choice(n_sides, size=int(rng.integers(1, 12)), replace=False)
        counts = rng.integers(1, 5, len(sides))
        perm = rng.permutation(len(sides))
        block = torch.zeros(n_sides, dtype=torch.int64)
        total = int(counts.sum())
        p_ = torch.zeros(total, dtype=torch.int64)
        pos = 0
        for j in perm:  # the lanes' atomicAdd order
            sd, c = int(sides[j]), int(counts[j])
            block[sd] = (pos << 32) | c
            for k in range(c):
                tag += 1
                p_[pos + k] = tag
                want[sd].append(tag)
            pos += c
        n_ = (p_ % 7).to(torch.int32)
        s_ = (p_ % 3).to(torch.int8)
        m_sid, m_ptr, m_n, m_st, merged = merge_requery_round(m_sid, m_ptr, m_n, m_st, block, p_, n_, s_, n_sides)
        blk, ptr, nn, st = merged
        for sd in range(n_sides):
            start, cnt = int(blk[sd]) >> 32, int(blk[sd]) & 0xFFFFFFFF
            got = ptr[start:start + cnt].tolist()
            assert got == want[sd], (rnd, sd)
            assert nn[start:start + cnt].tolist() == [t % 7 for t in want[sd]]
            assert st[start:start + cnt].tolist() == [t % 3 for t in want[sd]]
