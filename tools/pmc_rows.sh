#!/bin/bash
# SQ counter passes over the rows-mode bench (each its own run).  usage: pmc_rows.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
k=0
for P in "$P1" "$P2"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_pmc$k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --batches 1 "$@" > gpurun_out/${TAG}_pmc$k.log 2>&1 || { echo "pass $k rc=$?"; tail -5 gpurun_out/${TAG}_pmc$k.log; exit 1; }
  f=$(find gpurun_out/${TAG}_pmc$k -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void sst::", "").replace("sst::", "")
    if "k_rows" not in k and "k_explain" not in k and "k_is_valid" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    cnt = max(n[(k, c)] for c in d)
    print(k, " ".join(f"{c}={v / cnt:.3g}" for c, v in sorted(d.items())))
PY
done
