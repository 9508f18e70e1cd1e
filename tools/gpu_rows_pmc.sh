#!/bin/bash
# Counter passes (tools/pmc_groups.txt, one rocprofv3 --pmc pass per group,
# kernel trace only) over bench.py --a8-source rows, for this tree's library
# and each variant build/ab/NAME.so; per-kernel summaries gpurun_out/TAG_V_pmc.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for v in main "$@"; do
  if [ $v = main ]; then unset SST_LIBRARY; else export SST_LIBRARY=$PWD/build/ab/$v.so; fi
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${v}_p$i -o pmc -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --a8-source rows > gpurun_out/${TAG}_${v}_p$i.log 2>&1
    rc=$?; echo "[$v pmc $i] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done < tools/pmc_groups.txt
  python3 tools/pmc_summary.py gpurun_out/${TAG}_${v}_pmc.json gpurun_out/${TAG}_${v}_p* > gpurun_out/${TAG}_${v}_pmc.txt 2>&1
  grep rows gpurun_out/${TAG}_${v}_pmc.txt
done
