#!/bin/bash
# rocprofv3 kernel stats of config 5 at N spectra (the frontier's kernels), all stages.  usage: gpu_frontier_prof.sh TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-frprof}; N=${2:-16384}
export PYTHONHASHSEED=0
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o trace -- python3 tools/pipeline_bench.py --spectra $N --cpu-baseline-s 0 > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}.err; exit $rc; }
find gpurun_out/${TAG}_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
python3 - gpurun_out/${TAG}_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} total {float(r["TotalDurationNs"])/1e6:10.1f} ms avg {float(r["AverageNs"])/1e3:10.1f} us')
PY
