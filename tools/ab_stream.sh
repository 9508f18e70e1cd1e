cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 0 1 2 1 0 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --a7-stream $v > gpurun_out/ab_s$v.json 2>gpurun_out/ab_s$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab_s$v.json'));print($v, round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"
done
