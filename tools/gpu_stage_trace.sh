#!/bin/bash
# Config 5, stages 1-4 at N spectra (stage 5 on a few) under rocprofv3
# --kernel-trace --stats: the kernel stats CSV and, per kernel, every
# dispatch's duration in launch order (gpurun_out/TAG_dispatch.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-st}; N=${2:-100000}
export PYTHONHASHSEED=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o trace -- \
  python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --length-spectra ${LS:-8} \
  > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
python3 - gpurun_out/${TAG}_trace gpurun_out/${TAG}_dispatch.txt <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
per = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    per[r["Kernel_Name"].split("(")[0]].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
with open(sys.argv[2], "w") as o:
    for k, v in sorted(per.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        o.write(f"{k} calls={len(v)} total_us={sum(d for _, d in v):.1f}\n  " + " ".join(f"{d:.0f}" for _, d in v) + "\n")
print(open(sys.argv[2]).read()[:3000])
PY
