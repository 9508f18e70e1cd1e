#!/bin/bash
# GPU-box run: caller parity tests on the HIP engine, then the config-5
# pipeline harness (small, then full size).  usage: gpu_callers.sh TAG [spectra]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; N=${2:-100000}
timeout -k 10 600 python -u -m pytest tests/test_gpu_callers.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -20; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/pipeline_bench.py --spectra 2000 > gpurun_out/${TAG}_pipe_small.json 2> gpurun_out/${TAG}_pipe_small.err
rc=$?; echo "[pipe small] rc=$rc"; tail -c 1500 gpurun_out/${TAG}_pipe_small.json; tail -3 gpurun_out/${TAG}_pipe_small.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/pipeline_bench.py --spectra $N > gpurun_out/${TAG}_pipe.json 2> gpurun_out/${TAG}_pipe.err
rc=$?; echo "[pipe] rc=$rc"; tail -c 2500 gpurun_out/${TAG}_pipe.json; tail -3 gpurun_out/${TAG}_pipe.err
exit $rc
