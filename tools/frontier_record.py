#!/usr/bin/env python3
"""Join one matched stage-5 record (tools/gpu_frontier_record.sh TAG): the
kernel trace's per-kernel durations and dispatch counts, the FETCH_SIZE and
WRITE_SIZE passes of the same command (dispatch counts must agree), and the
run's node / group / edge counts (pipeline_bench's length stage) -> HBM bytes
per node measured by the counters against DESIGN §4's per-unit model, and the
kernels' rates.  gfx950: FETCH_SIZE reports half the bytes
(MI355X_MICROARCH.md), HBM bytes = 2 FETCH + WRITE (KB x 1024).

usage: frontier_record.py TAG   (reads gpurun_out/TAG_*; writes gpurun_out/TAG_record.json)"""
import csv
import glob
import json
import sys
from collections import defaultdict

KERNELS = ("k_lbf_groups", "k_lbf_nodes", "k_lbf_values", "k_lbf_roots", "k_lbf_setup", "k_lbf_out", "k_lbf_mark",
           "k_reach_rows", "k_reach_lowest")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("sst::", "")
    return n.split("<")[0]


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main():
    tag = sys.argv[1]
    base = f"gpurun_out/{tag}"
    trace = defaultdict(lambda: [0, 0.0])
    for f in glob.glob(f"{base}_trace/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if k in KERNELS:
                trace[k][0] += 1
                trace[k][1] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = defaultdict(lambda: [0, 0.0])
        for f in glob.glob(f"{base}_{c}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row["Kernel_Name"])
                if k in KERNELS and row["Counter_Name"] == c:
                    acc[k][0] += 1
                    acc[k][1] += float(row["Counter_Value"]) * 1024.0
        pmc[c] = acc
    runs = {n: last_json(f"{base}_{n}.json") for n in ("trace", "FETCH_SIZE", "WRITE_SIZE")}
    fr = [r["stages"]["length"]["frontier"] for r in runs.values()]
    assert all(f["nodes"] == fr[0]["nodes"] and f["chunks"] == fr[0]["chunks"] for f in fr), fr
    N, G, E = fr[0]["nodes"], fr[0]["groups"], fr[0]["edges"]
    # DESIGN §4's per-unit model for these counts, as pipeline_bench computes it now (not the copy in the run's
    # JSON: a re-join after a model change uses the current model); the trace run's kernel time
    sys.path.insert(0, "tools")
    from pipeline_bench import frontier_roofline
    model = frontier_roofline(fr[0], runs["trace"]["stages"]["length"]["kernels"])
    out = {"tag": tag, "spectra": runs["trace"]["spectra"], "nodes": N, "groups": G, "edges": E,
           "key_words": fr[0]["key_words"], "chunks": fr[0]["chunks"], "model": model, "kernels": {}}
    tot = {"s": 0.0, "hbm": 0.0, "algo": model["algorithmic_bytes"]}
    for k in KERNELS:
        if k not in trace:
            continue
        n_t, s_t = trace[k]
        n_f, b_f = pmc["FETCH_SIZE"].get(k, [0, 0.0])
        n_w, b_w = pmc["WRITE_SIZE"].get(k, [0, 0.0])
        assert n_f == n_t == n_w, (k, n_t, n_f, n_w)  # matched: the same dispatches in all three runs
        hbm = 2 * b_f + b_w
        out["kernels"][k] = {"dispatches": n_t, "s": s_t, "hbm_bytes": hbm, "hbm_GBps": hbm / s_t / 1e9 if s_t else 0,
                             "hbm_bytes_per_node": hbm / N}
        if k in ("k_lbf_groups", "k_lbf_nodes", "k_lbf_values"):
            tot["s"] += s_t
            tot["hbm"] += hbm
    out["frontier_band_kernels"] = {
        "s": tot["s"], "hbm_bytes": tot["hbm"], "hbm_bytes_per_node": tot["hbm"] / N,
        "model_bytes_per_node": tot["algo"] / N, "hbm_over_model": tot["hbm"] / tot["algo"],
        "hbm_GBps": tot["hbm"] / tot["s"] / 1e9, "frac_hbm_8TBps": tot["hbm"] / tot["s"] / 8e12,
        "model_GBps": tot["algo"] / tot["s"] / 1e9, "nodes_per_s": N / tot["s"],
        "random_lines_per_node": model["random_lines_per_node"],
        "random_lines_per_s": model["random_lines"] / tot["s"],
        "frac_random_line_rate": model["random_lines"] / tot["s"] / model["line_rate_peak"]}
    json.dump(out, open(f"{base}_record.json", "w"), indent=1)
    print(json.dumps(out["frontier_band_kernels"], indent=1))
    print({k: (v["dispatches"], round(v["s"], 3), round(v["hbm_bytes_per_node"], 1)) for k, v in out["kernels"].items()})


if __name__ == "__main__":
    main()
