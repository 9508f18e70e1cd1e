#!/bin/bash
# GPU-box check run: smoke, GPU parity tests, one short bench line (no CPU
# baseline).  Stops at the first step that ends in a fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-check}
shift
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a "gpurun_out/${TAG}_summary.log"
  tail -4 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gputests 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread "$@"
step bench 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline
