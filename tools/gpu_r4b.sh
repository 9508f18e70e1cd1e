#!/bin/bash
# Round 4: the device skeleton walk against the reference fixtures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline_device.py -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "skeleton_walk" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "PASSED|FAILED|ERROR|assert" gpurun_out/${TAG}_tests.log | head -40; tail -3 gpurun_out/${TAG}_tests.log; exit $rc
