#!/bin/bash
# config-1 same-box comparison of library variants: c1_variants2.sh NAME... (build/ab/NAME.so), interleaved x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for v in "$@"; do
  rm -rf gpurun_out/c1v_$v
  SST_LIBRARY=$PWD/build/ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1v_$v -o run -- python3 bench.py --workload config1 --steps 20 --no-cpu-baseline --no-validate > gpurun_out/c1v_$v.json 2> gpurun_out/c1v_$v.err || { echo "$v failed"; tail -3 gpurun_out/c1v_$v.err; exit 1; }
  f=$(find gpurun_out/c1v_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'k_explain_deferred' in r['Name']: print('$v', 'k_explain_deferred', round(float(r['AverageNs'])/1e3,1), 'us')"
done; done
