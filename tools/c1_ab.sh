#!/bin/bash
# Config-1 same-box A/B: this tree's library ("new") against build/ab/base.so,
# interleaved, rocprofv3 averages of the deferred kernel and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export SST_LIBRARY=$PWD/build/ab/base.so; else unset SST_LIBRARY; fi
  rm -rf gpurun_out/c1ab_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1ab_$v -o run -- python3 bench.py --workload config1 --steps 20 --no-cpu-baseline "$@" > gpurun_out/c1ab_$v.json 2> gpurun_out/c1ab_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/c1ab_$v.err; exit 1; }
  f=$(find gpurun_out/c1ab_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" gpurun_out/c1ab_$v.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = {r["Name"].split("(")[0].replace("void sst::", "").replace("sst::", ""): float(r["AverageNs"]) / 1e3
      for r in rows if "k_explain" in r["Name"] or "k_result_pack" in r["Name"]}
print(sys.argv[2], f"{d['value'] / 1e6:.1f} M/s", f"{d['ms_per_step'] * 1e3:.1f} us/step",
      " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items())), flush=True)
PY
done
