#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) over the config-5
# pipeline at 20 k spectra (stage 5 on one spectrum), then the per-kernel
# summary.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4p}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/pipeline_bench.py --spectra 20000 --warmup-spectra 16 --length-spectra 1 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i: $grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < tools/pmc_groups.txt
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"; grep -A12 "k_valid_alpha" gpurun_out/${TAG}_pmc.txt | head -30
