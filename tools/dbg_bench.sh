cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_pipeline_device.py tests/test_gpu_alpha.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/dbg0.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|Error|error" gpurun_out/dbg0.log | head -30
timeout -k 10 200 python -u bench.py --spectra 1500 --steps 4 --warmup 1 --no-cpu-baseline --a8-source queries > gpurun_out/dbg1.log 2>&1; echo "q rc=$?"; tail -3 gpurun_out/dbg1.log | cut -c1-400
timeout -k 10 200 python -u bench.py --spectra 1500 --steps 4 --warmup 1 --no-cpu-baseline --a8-source rows > gpurun_out/dbg3.log 2>&1; echo "rows rc=$?"; tail -3 gpurun_out/dbg3.log | cut -c1-400
SST_DEVICE=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --spectra 1200 --steps 4 --warmup 1 --batches 2 --no-cpu-baseline --a8-source queries > gpurun_out/dbg2.log 2>&1; echo "n2 rc=$?"; grep -v Warning gpurun_out/dbg2.log | grep -B2 -A12 "Traceback" | head -40
