#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over
# config 5 at N spectra (stage 5 on all of them: the frontier's kernels);
# summary per kernel in gpurun_out/TAG_pmc.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fpmc}; N=${2:-16000}
export PYTHONHASHSEED=0
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i: $grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < tools/pmc_groups.txt
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"
