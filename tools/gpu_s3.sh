#!/bin/bash
# DFS-kernel iteration: GPU tests (-k), config-1 A/B vs build/ab/base.so, phase clocks (build/ab/time.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; KEXPR=$2
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "$KEXPR" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
bash tools/c1_ab.sh || exit 1
SST_LIBRARY=$PWD/build/ab/time.so timeout -k 10 300 python -u tools/c1_time.py
