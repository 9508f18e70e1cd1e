#!/bin/bash
# PMC passes over stage 5 (the reach-mode length-bound replay) on a
# 128-spectrum sample: instruction mix and wait counters of k_length_exact.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4lb}
i=0
head -3 tools/pmc_groups.txt | while read -r grp; do
  i=$((i+1))
  timeout -s KILL 280 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/pipeline_bench.py --spectra 512 --warmup-spectra 16 --length-spectra 128 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"; grep "k_length_exact" gpurun_out/${TAG}_pmc.txt | cut -c1-900
