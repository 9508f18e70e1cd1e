#!/bin/bash
# One GPU call: smoke, the GPU parity tests, the default bench line, and the
# same bench under rocprofv3 --kernel-trace --stats.  Stops at the first step
# that faults / aborts / times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-val}
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed $?; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo "[smoke] ok"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread --durations=10 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -15 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "[bench] rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
rc=$?; echo "[rocprof] rc=$rc"; find gpurun_out/${TAG}_prof -name "*stats*"
exit $rc
