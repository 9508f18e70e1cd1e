#!/bin/bash
# Same-box A/B of environment variants of one build: bench lines (no CPU
# baseline, --no-validate for diagnostic variants) per "NAME=VAR=VALUE" arg,
# interleaved over 3 rounds.  usage: ab_env.sh TAG base SST_PACK_DBG=1 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
for r in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 $BENCH_EXTRA > gpurun_out/${TAG}_r$r.json 2>gpurun_out/${TAG}_r$r.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_r$r.json'));print('$v', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"
  done
done
