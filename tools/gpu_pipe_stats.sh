#!/bin/bash
# Config 5 at N spectra, every stage, under rocprofv3 --kernel-trace --stats:
# the kernel stats CSV of the whole run.  usage: gpu_pipe_stats.sh TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pst}; N=${2:-100000}
export PYTHONHASHSEED=0
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- \
  python3 tools/pipeline_bench.py --spectra $N --warmup-spectra 16 --cpu-baseline-s 0 > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}.err | cut -c1-300
[ $rc -ne 0 ] && exit $rc
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
head -12 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-160
