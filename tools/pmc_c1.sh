#!/bin/bash
# Config-1 counter passes (the config-1 line's roofline.traffic):
# FETCH_SIZE and WRITE_SIZE in their own rocprofv3 --pmc runs (kernel trace
# only), then the SQ groups of tools/pmc_groups.txt, over a short config-1 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-c1pmc}
BENCH="bench.py --workload config1 --steps 5 --warmup 1 --no-cpu-baseline"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 $BENCH > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i: $grp] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done < tools/pmc_groups.txt
python3 tools/pmc_summary.py --traffic gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"; grep -E "k_explain_deferred|k_explain_scan|k_result_pack" gpurun_out/${TAG}_pmc.txt | cut -c1-400
