#!/bin/bash
# N=2 rehearsal of the multi-rank bench on ONE GPU (gloo backend, both ranks
# on device 0), with the (default) gather of all results to rank 0 and without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${1:-mr}
for g in "" "--no-gather"; do
  SST_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --spectra 4000 $g \
    > gpurun_out/${TAG}_n2${g}.json 2> gpurun_out/${TAG}_n2${g}.err
  rc=$?; echo "[n2 $g] rc=$rc"; tail -c 600 gpurun_out/${TAG}_n2${g}.json; echo
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_n2${g}.err; exit $rc; }
done
exit 0
