#!/bin/bash
# Frontier A/B: its parity tests on this tree's library, then stage 5 at N
# spectra for this tree and each variant (build/ab/NAME.so), twice, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
export PYTHONHASHSEED=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_length_frontier.py > gpurun_out/${TAG}_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_t.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in main "$@"; do
    if [ $v = main ]; then unset SST_LIBRARY; else export SST_LIBRARY=$PWD/build/ab/$v.so; fi
    timeout -k 10 300 python -u tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0 ${AB_ARGS:-} > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 gpurun_out/${TAG}_${v}_$r.err; exit $rc; }
    python3 - gpurun_out/${TAG}_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
L = d["stages"]["length"]
print(sys.argv[2], "length", round(L["s"], 3), "s", L["kernels"], flush=True)
PY
  done
done
