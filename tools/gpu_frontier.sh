#!/bin/bash
# Stage-5 frontier engine: parity tests, then config 5 at N spectra.  usage: gpu_frontier.sh TAG [N] [tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fr}
N=${2:-4096}
TESTS=${3:-tests/test_gpu_length_frontier.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
fi
SST_PIPE_PROGRESS=1 timeout -k 10 900 python -u tools/pipeline_bench.py --spectra $N > gpurun_out/${TAG}_pipe.json 2> gpurun_out/${TAG}_pipe.err
rc=$?; echo "pipe rc=$rc"; tail -4 gpurun_out/${TAG}_pipe.err
[ $rc -ne 0 ] && exit $rc
python3 - gpurun_out/${TAG}_pipe.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("total", round(d["total_s"], 3), {k: round(v["s"], 3) for k, v in d["stages"].items()})
L = d["stages"]["length"]
print("length", L["lb_status"], L["frontier"], L.get("cpu_baseline"), L["replay_nodes"])
PY
