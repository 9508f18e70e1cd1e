#!/bin/bash
# Stage 5 at N spectra for several frontier workspace sizes (GiB; smaller =
# smaller chunks of queries and hash tables).  usage: gpu_frontier_ws.sh TAG N GB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
export PYTHONHASHSEED=0
for gb in "$@"; do
  timeout -k 10 300 python -u tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0 \
    --frontier-workspace-gb $gb > gpurun_out/${TAG}_$gb.json 2> gpurun_out/${TAG}_$gb.err
  rc=$?; [ $rc -ne 0 ] && { echo "$gb rc=$rc"; tail -3 gpurun_out/${TAG}_$gb.err; exit $rc; }
  python3 - gpurun_out/${TAG}_$gb.json $gb <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
L = d["stages"]["length"]
print(sys.argv[2], "GiB: length", round(L["s"], 3), "s", L.get("frontier"), flush=True)
PY
done
