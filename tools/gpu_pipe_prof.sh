#!/bin/bash
# Config 5: the 100 k-spectrum device-resident pipeline line, its rocprofv3
# kernel stats, and PMC passes (one counter group per run, kernel trace only)
# over a 20 k-spectrum run.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-c5}; N=${2:-100000}; PMC=${3:-1}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "gpurun_out/${TAG}_${name}.log" | cut -c1-800
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
SST_PIPE_PROGRESS=1 step pipe 600 python -u tools/pipeline_bench.py --spectra $N --warmup-spectra 64 --length-spectra ${LS:-256}
SST_PIPE_PROGRESS=1 step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o trace -- python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 64 --length-spectra ${LS:-256}
find gpurun_out/${TAG}_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
[ "$PMC" = "0" ] && exit 0
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/pipeline_bench.py --spectra 20000 --warmup-spectra 16 --length-spectra 16 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i: $grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < tools/pmc_groups.txt
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"
