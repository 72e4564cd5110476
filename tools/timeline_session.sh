set -u
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/tl_h; mkdir -p $O
cd /tmp
for spp in 64 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/s$spp -o run --output-format csv -- python3 $R/tools/frame_loop.py 60 overlap 8 $spp > $O/s$spp.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/full -o run --output-format csv -- python3 $R/tools/frame_loop.py 40 overlap 1 64 > $O/full.log 2>&1 || exit 1
for d in s64 s1 full; do f=$(find $O/$d -name '*kernel_trace.csv' | head -1); echo "== $d"; python3 $R/tools/trace_timeline.py $f 5; done > $O/timelines.txt
echo ok
