#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: mean counter value per dispatch, per kernel.

usage: pmc_summary.py [--traffic TRAFFIC.json] OUT.json DIR [DIR ...]
       (DIRs hold pmc_counter_collection.csv; TRAFFIC.json = {kernel: HBM bytes per launch})

FETCH_SIZE / WRITE_SIZE are KB; on gfx950 FETCH_SIZE reports half the bytes
(MI355X_MICROARCH.md, HBM/rocprofv3 section), so hbm_bytes = 2*FETCH + WRITE.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def bench_name(k):
    """sst::k_explain_scan<true> -> k_explain_scan (the names bench.py reports)."""
    k = k.replace("sst::", "")
    return k.split("<")[0] if k.startswith(("k_explain_scan", "k_step")) else k


def main():
    traffic_out = None
    if sys.argv[1] == "--traffic":
        traffic_out = sys.argv[2]
        del sys.argv[1:3]
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"].split("(")[0]
                    k = k.replace("void ", "")
                    if not k.startswith(("sst::", "k_")):  # engine kernels, tools/pmc_calib kernels
                        continue
                    c = row["Counter_Name"]
                    acc[k][c] += float(row["Counter_Value"])
                    cnt[k][c].add(row["Dispatch_Id"])
    res = {}
    for k, cs in acc.items():
        r = {c: v / max(1, len(cnt[k][c])) for c, v in cs.items()}
        r["dispatches"] = max(len(s) for s in cnt[k].values())
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["hbm_bytes"] = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024.0
        if "SQ_WAVES" in r and "SQ_INSTS_VALU" in r:
            r["valu_per_wave"] = r["SQ_INSTS_VALU"] / max(1.0, r["SQ_WAVES"])
        res[k] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    if traffic_out:  # roofline.traffic of bench.py: HBM bytes per launch
        tr = {bench_name(k): r["hbm_bytes"] for k, r in res.items() if "hbm_bytes" in r}
        with open(traffic_out, "w") as fh:
            json.dump(tr, fh, indent=1, sort_keys=True)
    for k, r in sorted(res.items()):
        print(k, {c: round(v, 1) for c, v in r.items()})


if __name__ == "__main__":
    main()
