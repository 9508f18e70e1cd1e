#!/bin/bash
# Config-1 tail diagnostics on a DIAG build (build/ab/diag.so): the deferred
# kernel with roles switched off (SST_TAIL_DBG: 1 no SHALLOW role, 2 no deep /
# exact roles, 4 the deep roles' counting DFS only), rocprofv3 averages.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export SST_LIBRARY=$PWD/build/ab/diag.so
for v in 0 1 2 4 5; do
  export SST_TAIL_DBG=$v
  rm -rf gpurun_out/td_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/td_$v -o run -- python3 bench.py --workload config1 --steps 20 --no-cpu-baseline --no-validate > gpurun_out/td_$v.json 2> gpurun_out/td_$v.err || exit $?
  f=$(find gpurun_out/td_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
print('dbg $v', [(r['Name'].split('(')[0].replace('void ','').replace('sst::',''), round(float(r['AverageNs'])/1e3,1)) for r in csv.DictReader(open('$f')) if 'k_explain' in r['Name'] or 'k_result' in r['Name']])"
done
