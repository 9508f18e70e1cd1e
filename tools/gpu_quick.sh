#!/bin/bash
# GPU-box iteration run: the result-path GPU tests, one bench line (no CPU
# baseline) and the same bench under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-quick}
shift
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_results.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "[bench] rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
rc=$?; echo "[rocprof] rc=$rc"
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_kernel_stats.csv 2>/dev/null; cut -c1-160 gpurun_out/${TAG}_kernel_stats.csv | head -12
exit $rc
