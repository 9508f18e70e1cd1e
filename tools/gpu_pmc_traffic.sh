#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run, kernel
# trace only) over the config-3 bench lines: the default (k_step) and
# --a8-source rows; per-kernel HBM bytes per launch in gpurun_out/TAG_*_traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-tr}
for line in step rows; do
  extra=""; [ $line = rows ] && extra="--a8-source rows"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_${line}_$c -o pmc -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $extra > gpurun_out/${TAG}_${line}_$c.log 2>&1
    rc=$?; echo "[$line $c] rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
  python3 tools/pmc_summary.py --traffic gpurun_out/${TAG}_${line}_traffic.json gpurun_out/${TAG}_${line}_pmc.json \
    gpurun_out/${TAG}_${line}_FETCH_SIZE gpurun_out/${TAG}_${line}_WRITE_SIZE > gpurun_out/${TAG}_${line}_pmc.txt 2>&1
  echo "[$line summary] rc=$?"; cat gpurun_out/${TAG}_${line}_traffic.json
done
