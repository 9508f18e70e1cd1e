#!/bin/bash
# k_valid_alpha: its parity tests, then an A/B of library variants on the
# config-5 pipeline (stages 1-4 at N spectra).  usage: gpu_valid_alpha.sh VARIANT...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export PYTHONHASHSEED=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_alpha.py tests/test_gpu_pipeline_device.py tests/test_gpu_callers.py > gpurun_out/va_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/va_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_pipe.sh "$@"
