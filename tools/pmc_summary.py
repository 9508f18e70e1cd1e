#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: mean counter value per dispatch, per kernel.

usage: pmc_summary.py OUT.json DIR [DIR ...]   (DIRs hold pmc_counter_collection.csv)

FETCH_SIZE / WRITE_SIZE are KB; on gfx950 FETCH_SIZE reports half the bytes
(MI355X_MICROARCH.md, HBM/rocprofv3 section), so hbm_bytes = 2*FETCH + WRITE.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"].split("(")[0]
                    if not k.startswith(("sst::", "void sst::")):
                        continue
                    k = k.replace("void ", "")
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
    for k, r in sorted(res.items()):
        print(k, {c: round(v, 1) for c, v in r.items()})


if __name__ == "__main__":
    main()
