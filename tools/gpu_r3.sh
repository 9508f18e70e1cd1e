#!/bin/bash
# Round-3 GPU run: smoke, the GPU test suite, the default bench line and a
# rocprofv3 kernel-trace summary of the bench.  Each GPU step has its own time
# limit; the script stops at the first fault / abort / timeout.
# usage: tools/gpu_r3.sh TAG [tests|notests] [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
MODE=${2:-tests}
KEXPR=${3:-}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -4 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
if [ "$MODE" = tests ]; then
  if [ -n "$KEXPR" ]; then
    step gputests 1100 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=12 -k "$KEXPR"
  else
    step gputests 1100 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=12
  fi
fi
step bench 400 python -u bench.py
cp gpurun_out/${TAG}_bench.log gpurun_out/${TAG}_bench.json
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --no-cpu-baseline --steps 20
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
echo done
