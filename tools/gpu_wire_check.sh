#!/bin/bash
# Wire format v4 on the GPU: the device packer's tests, its standalone time on
# the config-3 result (events, then a rocprofv3 kernel summary), and the N=2
# gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_results.py > gpurun_out/w4_tests.log 2>&1 || { tail -40 gpurun_out/w4_tests.log; exit 1; }
tail -3 gpurun_out/w4_tests.log
timeout -k 10 120 python tools/wire_bench.py > gpurun_out/wb.json 2> gpurun_out/wb.err || { tail -5 gpurun_out/wb.err; exit 1; }
cat gpurun_out/wb.json
rm -rf gpurun_out/wb_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wb_prof -o run -- python3 tools/wire_bench.py > gpurun_out/wb_prof.json 2> gpurun_out/wb_prof.err || { tail -5 gpurun_out/wb_prof.err; exit 1; }
bash tools/gpu_multi_rehearsal.sh w4 || exit 1
