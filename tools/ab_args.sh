#!/bin/bash
# Same-box A/B of bench.py argument variants: ab_args.sh TAG "args A" "args B" ...
# (3 interleaved rounds, no CPU baseline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
for r in 1 2 3; do
  k=0
  for v in "$@"; do
    k=$((k+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 $v > gpurun_out/${TAG}_r${r}_$k.json 2>gpurun_out/${TAG}_r${r}_$k.err || exit $?
    python -c "import json;L=[l for l in open('gpurun_out/${TAG}_r${r}_$k.json') if l.startswith('{')][0];d=json.loads(L);print('[$v]', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"
  done
done
