"""Run in a child process by test_gpu_engine.py::test_exact_retry_ladder with
SST_EXACT_HASH_CAP0=16: every budget-binding window of the exact path then
exhausts its first per-lane memo, and the settle's retry ladder (8x the memo
over 8x fewer lanes: 2048 -> 256 -> 64 lanes, the last rung a deferred-kernel
workgroup with idle waves) must still give the oracle's answers."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import _oracle as oracle  # noqa: E402
import test_gpu_engine as T  # noqa: E402
from conftest import load_golden  # noqa: E402
from spectrseqtools_amd import _native  # noqa: E402


def main():
    assert os.environ.get("SST_EXACT_HASH_CAP0") == "16"
    g = load_golden("alphabet.json")
    ms = sorted({r["tolerated_integer_masses"] for r in g["rows"]} | {0})
    eng = _native.get_engine(0)
    dev = _native.DeviceTable.build(ms, max(ms) * 35, 32, engine=eng)
    host = oracle.build_table(ms, max(ms) * 35, 32)
    rng = np.random.default_rng(19)
    n = 0
    for L in (4, 3, 2):  # the heaviest memo first: the ladder starts at 16 entries per lane
        seqs = [rng.choice([305042, 306026, 329053, 345048], L) for _ in range(10)]
        masses = np.array([s.sum() * 1e-3 for s in seqs])
        max_len = int(masses.max() / 1e-3 / 305042)
        is_mod, caps = T._alph(ms, max_len)
        T._check_explain(dev, host, ms, is_mod, caps, masses, None, round(0.5 * L), True, tol=10e-6)
        n += len(masses)
    print(f"exact retry ladder ok: {n} queries")


if __name__ == "__main__":
    main()
