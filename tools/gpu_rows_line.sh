#!/bin/bash
# The config-3 bench lines: --a8-source rows and the default, each 30 steps
# (JSON lines into gpurun_out/TAG_rows.json / TAG_default.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-bl}
timeout -k 10 400 python bench.py --steps 30 --a8-source rows > gpurun_out/${TAG}_rows.json 2> gpurun_out/${TAG}_rows.err
rc=$?; echo "rows rc=$rc"; tail -c 600 gpurun_out/${TAG}_rows.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 30 > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err
rc=$?; echo "default rc=$rc"; tail -c 600 gpurun_out/${TAG}_default.json; exit $rc
