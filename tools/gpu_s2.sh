#!/bin/bash
# Session-2 GPU run: the GPU suite (optionally -k), then the config-1 same-box
# A/B against build/ab/base.so (tools/c1_ab.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-s2}; KEXPR=${2:-}
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "$KEXPR" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?; echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
bash tools/c1_ab.sh
