#!/bin/bash
# A/B of bench argument sets on one box: ab_bench_args.sh TAG "args A" "args B" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  k=0
  for a in "$@"; do
    k=$((k+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 $a > gpurun_out/${TAG}_$k.json 2>gpurun_out/${TAG}_$k.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_$k.json'));print('[$a]', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3))"
  done
done
