#!/bin/bash
# Same-box rocprofv3 A/B of two builds: this tree's libsstgpu.so ("new")
# against tools/libsst_base.so ("base"), interleaved; per-kernel average
# durations of the bench's kernels.  usage: ab_prof.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export SST_LIBRARY=$PWD/tools/libsst_base.so; else unset SST_LIBRARY; fi
  rm -rf gpurun_out/pkp_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pkp_$v -o run -- python3 bench.py --steps 40 --no-cpu-baseline "$@" > gpurun_out/pkp_$v.json 2> gpurun_out/pkp_$v.err || exit $?
  f=$(find gpurun_out/pkp_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" gpurun_out/pkp_$v.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
ks = {r["Name"].split("(")[0].replace("void sst::", ""): float(r["AverageNs"]) / 1e3 for r in rows
      if "k_is_valid" in r["Name"] or "k_explain" in r["Name"] or "k_result_pack" in r["Name"]}
print(sys.argv[2], f"{d['value'] / 1e9:.2f} G/s", f"{d['ms_per_step'] * 1e3:.1f} us/step",
      " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items())), flush=True)
PY
done
