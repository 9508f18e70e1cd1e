#!/bin/bash
# GPU-box measurement run: bench line, then the same command under rocprofv3
# --kernel-trace --stats (no PMC here; counters run in their own passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
shift
ARGS="$@"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py $ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "[bench] rc=$rc"; tail -c 3000 gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
rc=$?; echo "[rocprof] rc=$rc"
find gpurun_out/${TAG}_prof -name "*stats*" | head
