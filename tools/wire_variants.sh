cd /root/repo; export TMPDIR=/tmp
for v in "" build/ab/nolist.so build/ab/noC.so build/ab/noF.so ""; do
  if [ -n "$v" ]; then export SST_LIBRARY=$PWD/$v; else unset SST_LIBRARY; fi
  echo -n "${v:-base} "; timeout -k 10 120 python tools/wire_bench.py --no-check 2> gpurun_out/wv.err | cut -c1-60 || { tail -3 gpurun_out/wv.err; exit 1; }
done
