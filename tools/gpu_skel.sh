#!/bin/bash
# The skeleton stage: its parity tests, then the config-5 pipeline (stages
# 1-4 at N spectra) under rocprofv3 --kernel-trace (tools/gpu_stage_trace.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export PYTHONHASHSEED=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_explain_alpha.py tests/test_gpu_pipeline_device.py tests/test_gpu_callers.py > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_stage_trace.sh ${1:-sk}
