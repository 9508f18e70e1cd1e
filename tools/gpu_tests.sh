#!/bin/bash
# GPU parity tests only (optionally a -k filter): gpu_tests.sh TAG [pytest args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -15; tail -3 gpurun_out/${TAG}_tests.log; exit $rc
