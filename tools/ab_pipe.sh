#!/bin/bash
# A/B of library variants on the config-5 pipeline (stages 1-4 at N spectra,
# stage 5 on a few): per variant, every stage's kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
N=${N:-100000}
for v in "$@"; do
  SST_LIBRARY=build/ab/$v.so timeout -k 10 300 python -u tools/pipeline_bench.py --spectra $N --warmup-spectra 16 \
    --length-spectra 8 > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
line = [l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")][-1]
d = json.loads(line)
ks = {k: round(x[0], 2) for st in d["stages"].values() for k, x in st.get("kernels", {}).items()}
print(v, {s: round(x["s"], 4) for s, x in d["stages"].items()}, ks, flush=True)
PY
done
