"""Time sst_wire_pack alone on the config-3 step result (1 GPU): the step
once, then K packs of its result into a buffer of the agreed size, bracketed
by HIP events on the engine stream.  Prints one JSON line (pack us, wire
bytes, list entries, and the A7 / A8 / pair-hit counts it packed).

    python tools/wire_bench.py [--spectra 10000] [--iters 50]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spectra", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-check", action="store_true", help="skip decoding (experimental builds)")
    args = ap.parse_args()
    import torch

    import bench
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE
    from spectrseqtools_amd.mass_table import DynamicProgrammingTable, SequenceInformation
    from spectrseqtools_amd.parallel import wire_unpack, wire_used_bytes

    engine = _native.get_engine(0)
    dev_t = torch.device("cuda", 0)
    seq = SequenceInformation(max_len=20, su_mass=6500.0, obs_mass=6500.0, modification_rate=0.5)
    dp = DynamicProgrammingTable(EXPLANATION_MASSES, compression_rate=32, tolerance=MATCHING_THRESHOLD,
                                 precision=TOLERANCE, seq=seq, engine=engine)
    A = round(seq.modification_rate * seq.max_len)
    tdev = dp.device_table
    wl = bench.build_workload(args.spectra, 1234, dp)
    n7, n8 = len(wl["a7_mass"]), len(wl["a8_mass"])
    obs = torch.from_numpy(wl["obs"]).to(dev_t)
    a8m = torch.from_numpy(wl["a8_mass"]).to(dev_t)
    a8t = torch.from_numpy(wl["a8_thr"]).to(dev_t)
    out7 = torch.empty(n7, dtype=torch.int8, device=dev_t)
    torch.cuda.synchronize()
    r = tdev.step_device(obs.data_ptr(), len(wl["obs"]), wl["shifts"], out7.data_ptr(), a8m.data_ptr(),
                         a8t.data_ptr(), n8, dp.tolerance, dp.precision, A)
    r.settle()
    fixed = r.wire_pack(out7.data_ptr(), n7)
    buf = torch.empty(fixed + 8 * (n7 + n8), dtype=torch.uint8, device=dev_t)
    torch.cuda.synchronize()
    ext = torch.cuda.ExternalStream(engine.stream, device=dev_t)
    for _ in range(3):
        r.wire_pack(out7.data_ptr(), n7, buf.data_ptr(), buf.numel())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext)
    for _ in range(args.iters):
        r.wire_pack(out7.data_ptr(), n7, buf.data_ptr(), buf.numel())
    e1.record(ext)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / args.iters
    host = buf.cpu().numpy()
    used = wire_used_bytes(host)
    h = host[:128].view(np.uint64)
    if not args.no_check:
        _v, st, _hits, _pay = wire_unpack(host[:used], tdev.pair_records())
        r.fetch_device()
        assert np.array_equal(st, r.status)
    print(json.dumps({"pack_us": us, "wire_bytes": used, "fixed_bytes": fixed, "list_entries": int(h[9]),
                      "a7": n7, "a8": n8, "pair_hits": int(h[3]), "explicit_hits": int(h[4]), "w": int(h[8]),
                      "spectra": args.spectra}))


if __name__ == "__main__":
    main()
