#!/bin/bash
# GPU-box validation run: smoke, GPU parity tests.  Stops at the first step that
# ends in a fault/abort/timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a "gpurun_out/${TAG}_summary.log"
  tail -3 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gputests 1200 python -m pytest tests -x -q -m gpu -p no:cacheprovider --durations=8
