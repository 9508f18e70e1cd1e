#!/bin/bash
# The rows line's record (bench.py --a8-source rows): FETCH_SIZE / WRITE_SIZE
# passes (one counter per rocprofv3 run, kernel trace only) -> per-kernel HBM
# bytes per launch; the bench line itself (CPU leg included); the same bench
# under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rrec}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_$c -o pmc -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --a8-source rows > gpurun_out/${TAG}_$c.log 2>&1
  rc=$?; echo "[$c] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py --traffic gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_pmc.json \
  gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[summary] rc=$?"; cat gpurun_out/${TAG}_traffic.json
timeout -k 10 400 python3 bench.py --a8-source rows > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- \
  python3 bench.py --a8-source rows --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo "[rocprof] rc=$?"
