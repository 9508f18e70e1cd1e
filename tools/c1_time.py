#!/usr/bin/env python3
"""Phase clocks of the deferred kernel's deep role on the config-1 step (a
-DSST_DIAG_TIME build, SST_LIBRARY=build/ab/time.so): per wave, s_memrealtime
(100 MHz) at entry, after staging, before the DFS, after it, after the payload
allocation, after the hit records, at exit; printed as percentiles relative
to the earliest entry."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    import bench
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, TOLERANCE, UNMODIFIED_BASES

    eng = _native.get_engine(0)
    lib = eng._lib
    seq = SequenceInformation(max_len=8, su_mass=0.0, obs_mass=0.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=10e-6, precision=TOLERANCE,
                                 seq=seq, engine=eng)
    dp.adapt_individual_modification_rates_by_alphabet_reduction(set(UNMODIFIED_BASES))
    tdev = dp.device_table
    mass, thr, mods = bench.config1_queries(200000, 0)
    dev = torch.device("cuda", 0)
    dm, dt, dmods = (torch.from_numpy(x).to(dev) for x in (mass, thr, mods))
    res = None
    for k in range(4):
        lib.sst_diag_time_clear()
        torch.cuda.synchronize()
        res = tdev.explain_device(dm.data_ptr(), dt.data_ptr(), len(mass), dp.tolerance, dp.precision, 0,
                                  d_mods=dmods.data_ptr(), reuse=res)
        res.settle()
        eng.synchronize()
    buf = np.zeros(1 << 20, np.uint64)
    lib.sst_diag_time_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    t = buf.reshape(-1, 8).astype(np.int64)
    t = t[t[:, 0] > 0]
    busy = t[t[:, 2] > 0]
    t0 = t[:, 0].min()
    print(f"waves entered {len(t)}, with a query {len(busy)}")
    names = ["entry", "staged", "dfs_start", "dfs_end", "alloc", "emit", "exit"]
    for k, nm in enumerate(names):
        v = (busy[:, k] - t0) / 100.0  # us
        print(f"{nm:10s} us after first entry: p0 {v.min():6.1f} p50 {np.median(v):6.1f} p90 {np.percentile(v, 90):6.1f}"
              f" max {v.max():6.1f}")
    for a, b in ((1, 2), (2, 3), (3, 4), (4, 5), (5, 6)):
        d = (busy[:, b] - busy[:, a]) / 100.0
        print(f"{names[a]}->{names[b]}: p50 {np.median(d):6.1f} p90 {np.percentile(d, 90):6.1f} max {d.max():6.1f} us")
    it = busy[:, 7]
    dfs = (busy[:, 3] - busy[:, 2]) / 100.0
    print(f"DFS loop iterations per wave (max over lanes): p50 {np.median(it):.0f} p90 {np.percentile(it, 90):.0f} "
          f"max {it.max()}; us per iteration p50 {np.median(dfs / np.maximum(it, 1)):.2f}")
    e = (t[:, 0] - t0) / 100.0
    print(f"all deep-role waves' entry: p50 {np.median(e):.1f} p90 {np.percentile(e, 90):.1f} max {e.max():.1f} us")


if __name__ == "__main__":
    main()
