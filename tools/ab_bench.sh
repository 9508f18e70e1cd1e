#!/bin/bash
# A/B timing on one GPU box: bench.py against several builds of libsstgpu.so
# (SST_LIBRARY), interleaved over rounds so box-to-box drift cancels.
# usage: [AB_ARGS=--no-validate] tools/ab_bench.sh ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    SST_LIBRARY=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 $AB_ARGS > gpurun_out/ab_${tag}_$r.json 2> gpurun_out/ab_${tag}_$r.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag round $r rc=$rc"; tail -3 gpurun_out/ab_${tag}_$r.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${tag}_$r.json')); print('$tag', $r, round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"
  done
done
