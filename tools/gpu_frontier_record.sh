#!/bin/bash
# One matched stage-5 record at N spectra: the kernel trace (rocprofv3
# --kernel-trace --stats) and the FETCH_SIZE / WRITE_SIZE passes (each its own
# run) of the SAME command -- same build, workspace, chunking -- joined by
# tools/frontier_record.py into gpurun_out/TAG_record.json.  usage: TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-frec}; N=${2:-16384}
export PYTHONHASHSEED=0
CMD="python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o trace -- $CMD > gpurun_out/${TAG}_trace.json 2> gpurun_out/${TAG}_trace.err
rc=$?; echo "[trace] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_trace.err; exit $rc; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 500 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_$c -o pmc -- $CMD > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  rc=$?; echo "[pmc $c] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$c.err; exit $rc; }
done
python3 tools/frontier_record.py $TAG > gpurun_out/${TAG}_record.txt 2>&1; rc=$?; cat gpurun_out/${TAG}_record.txt | tail -30; exit $rc
