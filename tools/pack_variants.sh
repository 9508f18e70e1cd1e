#!/bin/bash
# DIAGNOSTIC: k_result_pack variants (SST_PACK_DBG bits) under rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-pv}
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 4}; do
  SST_PACK_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_v$v -o trace -- python3 bench.py --no-cpu-baseline --no-validate --steps 20 > gpurun_out/${TAG}_v$v.log 2>&1
  rc=$?; echo "[variant $v] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_v$v.log; exit $rc; fi
  grep -h "k_result_pack\|k_explain_scan" gpurun_out/${TAG}_v$v/*kernel_stats.csv | cut -d, -f1-4
done
[ -n "$NO_PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_$c -o pmc -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/${TAG}_pmc_$c.log 2>&1
  rc=$?; echo "[pmc $c] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE
