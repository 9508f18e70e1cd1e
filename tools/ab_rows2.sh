#!/bin/bash
# rows-step line: GPU tests of the rows step, then same-box bench A/B of
# build/ab/base.so against this tree (interleaved x2) with rocprof kernel averages
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "rows or fullsize_rows" > gpurun_out/rows2_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/rows2_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in new base; do
  if [ $v = base ]; then export SST_LIBRARY=$PWD/build/ab/base.so; else unset SST_LIBRARY; fi
  rm -rf gpurun_out/rows2_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rows2_$v -o run -- python3 bench.py --a8-source rows --steps 20 --no-cpu-baseline > gpurun_out/rows2_$v.json 2> gpurun_out/rows2_$v.err || { echo "$v failed"; tail -3 gpurun_out/rows2_$v.err; exit 1; }
  f=$(find gpurun_out/rows2_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" gpurun_out/rows2_$v.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = {r["Name"].split("(")[0].replace("sst::", "").replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in rows if "rows" in r["Name"]}
print(sys.argv[2], f"{d['value'] / 1e9:.2f} G/s", f"{d['ms_per_step'] * 1e3:.1f} us/step", " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items())), flush=True)
PY
done; done
