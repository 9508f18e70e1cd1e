#!/bin/bash
# GPU-box counter passes (one rocprofv3 --pmc pass per counter group, kernel
# trace only, no sys/runtime trace) over a short bench run, plus the counter list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-pmc}
shift
export TMPDIR=/tmp
BENCH="bench.py --steps 5 --warmup 1 --no-cpu-baseline $@"
i=0

while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 $BENCH > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "[pmc $i: $grp] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < tools/pmc_groups.txt
python3 tools/pmc_summary.py --traffic gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.txt 2>&1
echo "[pmc summary] rc=$?"
# calibration of the counters for this kernel family's access widths
hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_calib_$c -o pmc -- ./tools/pmc_calib > gpurun_out/${TAG}_calib_$c.log 2>&1
  rc=$?; echo "[calib $c] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_calib.json gpurun_out/${TAG}_calib_FETCH_SIZE gpurun_out/${TAG}_calib_WRITE_SIZE > gpurun_out/${TAG}_calib.txt 2>&1
echo "[calib summary] rc=$?"
