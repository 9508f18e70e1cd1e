#!/bin/bash
# Round-5 checkpoint: the pipeline-device and masked-explain GPU tests, then
# config 5 at 100 k spectra (tools/gpu_pipe100k.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export PYTHONHASHSEED=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_explain_alpha.py tests/test_gpu_pipeline_device.py > gpurun_out/mid_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/mid_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_pipe100k.sh ${1:-p100k_r5}
