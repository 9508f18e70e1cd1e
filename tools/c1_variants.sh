#!/bin/bash
# Same-box rocprofv3 comparison of several builds on the config-1 workload:
# c1_variants.sh LIB... ("tree" = this tree's libsstgpu.so), interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for round in 1 2; do for v in "$@"; do
  if [ "$v" = tree ]; then unset SST_LIBRARY; else export SST_LIBRARY=$PWD/$v; fi
  tag=c1v_$(basename "$v" .so)
  rm -rf gpurun_out/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 bench.py --workload config1 --steps 20 --no-cpu-baseline > gpurun_out/$tag.json 2> gpurun_out/$tag.err || exit $?
  python3 - "$(find gpurun_out/$tag -name '*kernel_stats.csv' | head -1)" gpurun_out/$tag.json "$v" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {r["Name"].split("(")[0].replace("void sst::", "").replace("sst::", ""): float(r["AverageNs"]) / 1e3
      for r in rows if "k_explain" in r["Name"] or "k_result_pack" in r["Name"]}
print(sys.argv[3], f"{d['value'] / 1e6:.1f} M/s", f"{d['ms_per_step'] * 1e3:.1f} us/step",
      " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items())), flush=True)
PY
done; done
