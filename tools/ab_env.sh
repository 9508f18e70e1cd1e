#!/bin/bash
# A/B of environment settings on one box (same build), interleaved:
# ab_env.sh TAG ROUNDS "ENV=1 ..." "ENV=0 ..."   (use "-" for no setting)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  k=0
  for e in "$@"; do
    k=$((k+1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 $AB_ARGS > gpurun_out/${TAG}_$k.json 2>gpurun_out/${TAG}_$k.err || { echo "[$e] failed"; tail -3 gpurun_out/${TAG}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_$k.json'));print('[$e]', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"
  done
done
