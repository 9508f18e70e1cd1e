#!/bin/bash
# Quick GPU check: parity tests, then N bench lines (no CPU baseline).
# usage: ab_quick.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 "$@" > gpurun_out/${TAG}_b$k.json 2>gpurun_out/${TAG}_b$k.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$k.json'));print('$TAG', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3))"
done
