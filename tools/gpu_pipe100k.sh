#!/bin/bash
# Config 5 at N spectra (default 100 000), every stage on the device, stage-5 CPU baseline.  usage: gpu_pipe100k.sh TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-p100k}
N=${2:-100000}
export PYTHONHASHSEED=0  # the skeleton walk follows the interpreter's set order: one seed, reproducible runs
SST_PIPE_PROGRESS=1 timeout -k 10 1000 python -u tools/pipeline_bench.py --spectra $N > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
rc=$?; echo "pipe rc=$rc"; grep -v "skeleton walk\] launch" gpurun_out/${TAG}.err | tail -12
[ $rc -ne 0 ] && exit $rc
python3 - gpurun_out/${TAG}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("total", round(d["total_s"], 3), "peaks/s", round(d["peaks_per_s"]), {k: round(v["s"], 3) for k, v in d["stages"].items()})
L = d["stages"]["length"]
print("length", L["lb_status"], L["frontier"], L.get("cpu_baseline"), L["replay_nodes"], L["kernels"])
PY
