#!/bin/bash
# GPU-box run of the config-1 DFS workload: bench line, then rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload config1 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "[bench] rc=$rc"; tail -c 2500 gpurun_out/${TAG}_bench.json; tail -5 gpurun_out/${TAG}_bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --workload config1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
rc=$?; echo "[rocprof] rc=$rc"
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_kernel_stats.csv 2>/dev/null; cut -c1-150 gpurun_out/${TAG}_kernel_stats.csv | head -12
exit $rc
