#!/bin/bash
# Rows-step A/B (bench.py --a8-source rows): the rows parity tests on this
# tree's library, then the bench for this tree and each variant
# (build/ab/NAME.so), interleaved over rounds; a variant named prof* is a
# phase-clock build (SST_ROWS_PROF): its printed clock line is kept.
# usage: tools/gpu_rows_ab.sh TAG ROUNDS variant...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py \
  tests/test_gpu_fullsize.py -k "rows" > gpurun_out/${TAG}_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_t.log; [ $rc -ne 0 ] && exit $rc
for r in $(seq 1 $R); do
  for v in main "$@"; do
    if [ $v = main ]; then unset SST_LIBRARY; else export SST_LIBRARY=$PWD/build/ab/$v.so; fi
    timeout -k 10 300 python -u bench.py --a8-source rows --no-cpu-baseline --steps 30 > gpurun_out/${TAG}_${v}_$r.out 2> gpurun_out/${TAG}_${v}_$r.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 gpurun_out/${TAG}_${v}_$r.err; exit $rc; }
    python3 - gpurun_out/${TAG}_${v}_$r.out $v <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith("{")][-1])
prof = [l for l in lines if l.startswith("rows prof")]
print(sys.argv[2], round(d["ms_per_step"] * 1e3, 1), "us/step", round(d["roofline"]["avg_launch_us"], 1), "us/launch",
      prof[-1] if prof else "", flush=True)
PY
  done
done
unset SST_LIBRARY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python $GRAFT_REPO_ROOT/bench.py --a8-source rows --no-cpu-baseline --steps 30 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.out 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 $GRAFT_REPO_ROOT/tools/kstats.py $(find $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1) 2>/dev/null | grep -i rows
exit 0
