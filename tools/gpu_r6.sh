#!/bin/bash
# Round 6 GPU check: selected parity tests, then config 5 at N spectra.
# usage: gpu_r6.sh TAG N "test files" ["-k expression"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r6}
N=${2:-0}
TESTS=${3:-}
KEXPR=${4:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -40; tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
fi
if [ "$N" != "0" ]; then
  PYTHONHASHSEED=0 SST_PIPE_PROGRESS=1 timeout -k 10 900 python -u tools/pipeline_bench.py --spectra $N > gpurun_out/${TAG}_pipe.json 2> gpurun_out/${TAG}_pipe.err
  rc=$?; echo "pipe rc=$rc"; tail -4 gpurun_out/${TAG}_pipe.err
  [ $rc -ne 0 ] && exit $rc
  python3 - gpurun_out/${TAG}_pipe.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("total", round(d["total_s"], 3), {k: round(v["s"], 3) for k, v in d["stages"].items()})
print("classify cpu", d["stages"]["classify"].get("cpu_baseline"))
print("stages1to4 cpu", d.get("cpu_baseline_stages1to4"))
L = d["stages"]["length"]
print("length", L["lb_status"], L["frontier"], L.get("cpu_baseline"))
PY
fi
