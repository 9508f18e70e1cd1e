#!/bin/bash
# Round 4: device pipeline tests selected by -k (default: the skeleton / length ones).
# A heartbeat file under gpurun_out/ shows a long single test is alive.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4b}; K=${2:-skeleton}; FILES=${3:-tests/test_gpu_pipeline_device.py}
( while sleep 50; do date +%s >> gpurun_out/${TAG}_heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 800 python -u -m pytest $FILES -v -p no:cacheprovider --timeout 170 --timeout-method thread -k "$K" --durations=8 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; kill $HB 2>/dev/null; echo "[tests] rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error:|^E  " gpurun_out/${TAG}_tests.log | head -60; tail -12 gpurun_out/${TAG}_tests.log; exit $rc
