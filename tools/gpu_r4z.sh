#!/bin/bash
# Round 4, end of session: smoke, the whole GPU suite (without -x: every
# failure listed), then the config-5 pipeline at 100 k spectra (stage 5 on a
# 256-spectrum sample) under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4z}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/${TAG}_${name}.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
( while sleep 50; do date +%s >> gpurun_out/${TAG}_heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
step gputests 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 170 --timeout-method thread --durations=12
kill $HB 2>/dev/null
export SST_PIPE_PROGRESS=1
step pipeprof 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_pipeprof -o trace -- python3 tools/pipeline_bench.py --spectra 100000 --warmup-spectra 64 --length-spectra 256
find gpurun_out/${TAG}_pipeprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_pipe_kernel_stats.csv \;
echo done
