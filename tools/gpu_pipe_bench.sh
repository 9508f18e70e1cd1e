#!/bin/bash
# Config-5 pipeline bench, device-resident then host-driven stages.  usage: gpu_pipe_bench.sh TAG [spectra]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pipe}
N=${2:-100000}
timeout -k 10 400 python -u tools/pipeline_bench.py --spectra $N > gpurun_out/${TAG}_dev.json 2> gpurun_out/${TAG}_dev.err
rc=$?; echo "device rc=$rc"; [ $rc -ne 0 ] && { tail -8 gpurun_out/${TAG}_dev.err; exit $rc; }
timeout -k 10 600 python -u tools/pipeline_bench.py --spectra $N --host-driven > gpurun_out/${TAG}_host.json 2> gpurun_out/${TAG}_host.err
rc=$?; echo "host rc=$rc"; [ $rc -ne 0 ] && { tail -8 gpurun_out/${TAG}_host.err; exit $rc; }
python3 - gpurun_out/${TAG}_dev.json gpurun_out/${TAG}_host.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(d["path"], f"total {d['total_s']:.3f}s peaks/s {d['peaks_per_s']:.3g} busy {d['gpu_busy_frac']:.2f}",
          {k: (round(v["s"], 3), round(v.get("gpu_busy_frac", 0), 2)) for k, v in d["stages"].items()},
          "alph", d["stages"]["fixpoint"]["distinct_alphabets"], "hist", d["stages"]["fixpoint"]["rounds_histogram"])
PY
