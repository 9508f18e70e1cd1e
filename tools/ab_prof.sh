#!/bin/bash
# Same-box rocprofv3 A/B of two builds: this tree's libsstgpu.so ("new")
# against tools/libsst_base.so ("base"), interleaved; per-kernel average
# durations of the bench's kernels.  usage: ab_prof.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export SST_LIBRARY=$PWD/tools/libsst_base.so; else unset SST_LIBRARY; fi
  rm -rf gpurun_out/pkp_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pkp_$v -o run -- python3 bench.py --steps 40 --no-cpu-baseline "$@" > gpurun_out/pkp_$v.json 2> gpurun_out/pkp_$v.err || exit $?
  f=$(find gpurun_out/pkp_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_is_valid|k_explain_scan" "$f" | cut -d, -f1-5
done
