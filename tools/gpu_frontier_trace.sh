#!/bin/bash
# Stage 5 at N spectra under rocprofv3 --kernel-trace: every frontier
# dispatch in order, summarised per chunk (kernel time per band and pass,
# the gaps between dispatches).  usage: gpu_frontier_trace.sh TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ftr}; N=${2:-16000}
export PYTHONHASHSEED=0
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o trace -- \
  python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0 > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/${TAG}.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
python3 - gpurun_out/${TAG}_trace gpurun_out/${TAG}_chunks.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sst::", ""))
              for r in csv.DictReader(open(f)))
rows = [r for r in rows if "lbf" in r[2]]
chunks, cur = [], None
for s, e, n in rows:
    if n == "k_lbf_setup":
        cur = []
        chunks.append(cur)
    if cur is not None:
        cur.append((s, e, n))
with open(sys.argv[2], "w") as o:
    for ci, ch in enumerate(chunks):
        span = (ch[-1][1] - ch[0][0]) / 1e6
        busy = sum(e - s for s, e, _ in ch) / 1e6
        kinds = {}
        for s, e, n in ch:
            k = n.split("<")[0]
            kinds[k] = kinds.get(k, 0) + (e - s) / 1e6
        print(f"chunk {ci}: span {span:.2f} ms busy {busy:.2f} ms " +
              " ".join(f"{k}={v:.2f}" for k, v in sorted(kinds.items())), file=o)
        band, line = 0, []
        for s, e, n in ch:
            if n.startswith("k_lbf_groups") or n.startswith("k_lbf_nodes") or n == "k_lbf_values":
                line.append(f"{n.split('<')[0][6:]}:{(e - s) / 1e3:.0f}")
        print("   us " + " ".join(line), file=o)
print(open(sys.argv[2]).read()[:6000])
PY
