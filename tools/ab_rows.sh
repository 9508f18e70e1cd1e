#!/bin/bash
# Rows-step A/B: the GPU rows tests on this tree's library, then a kernel-trace
# summary of the rows-mode bench for it and for each variant library given
# (build/ab/NAME.so from tools/build_variant.py; a variant may be diagnostic,
# its bench may then fail its result check).  usage: ab_rows.sh TAG [NAME ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_multirank.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_t.log
[ $rc -ne 0 ] && { grep -E "^E |Error" gpurun_out/${TAG}_t.log | head -20; exit $rc; }
for v in main "$@"; do
  if [ $v = main ]; then unset SST_LIBRARY; else export SST_LIBRARY=$PWD/build/ab/$v.so; fi
  rm -rf gpurun_out/${TAG}_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$v -o run -- python3 bench.py --steps 20 --no-cpu-baseline --a8-source rows > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
  rc=$?
  [ $rc -ge 124 ] && { echo "$v: rc=$rc, stopping"; exit $rc; }
  f=$(find gpurun_out/${TAG}_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" gpurun_out/${TAG}_$v.json $rc <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = {r["Name"].split("(")[0].replace("void sst::", "").replace("sst::", ""): float(r["AverageNs"]) / 1e3 for r in rows
      if "k_rows" in r["Name"]}
try:
    d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); head = f"{d['value'] / 1e9:.2f} G/s {d['ms_per_step'] * 1e3:.1f} us/step"
except Exception:
    head = f"bench rc={sys.argv[4]}"
print(sys.argv[2], head, " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items())), flush=True)
PY
done
