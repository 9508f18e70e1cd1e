#!/bin/bash
# Rows-step check: its GPU tests, a rows-mode bench line and a kernel-trace
# summary of it.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-rows}
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_multirank.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1 \
  && echo "tests ok" \
  && timeout -k 10 300 python -u bench.py --no-cpu-baseline --a8-source rows > gpurun_out/${TAG}_b.log 2>&1 \
  && echo "bench ok" && tail -1 gpurun_out/${TAG}_b.log | cut -c1-600 \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --no-cpu-baseline --a8-source rows --steps 20 > gpurun_out/${TAG}_p.log 2>&1 \
  && find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \; \
  && cut -d, -f1-8 gpurun_out/${TAG}_kernel_stats.csv | head -14
rc=$?
[ $rc -ne 0 ] && { echo "rc=$rc"; grep -E "FAIL|Error|error" gpurun_out/${TAG}_t.log | head -20; tail -5 gpurun_out/${TAG}_b.log 2>/dev/null; }
exit $rc
