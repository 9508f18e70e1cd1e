#!/bin/bash
# Round-3 end-of-session run: smoke, the whole GPU suite, the default bench
# line + rocprof stats, the config-1 line + rocprof stats, the config-5
# pipeline (100 k spectra).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-s4}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/${TAG}_${name}.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gputests 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=10
step bench 400 python -u bench.py
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --no-cpu-baseline --steps 20
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
step c1 400 python -u bench.py --workload config1
step c1prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c1prof -o trace -- python3 bench.py --workload config1 --no-cpu-baseline --steps 20
find gpurun_out/${TAG}_c1prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_c1_kernel_stats.csv \;
step pipe 600 python -u tools/pipeline_bench.py --spectra 100000
echo done
