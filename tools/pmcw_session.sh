set -u
for a in "fullo librtc.so" "fullo librtc_prevcull.so" "share4o librtc.so" "share4o librtc_nomerge.so"; do
  set -- $a
  bash tools/pmc_writes.sh $1 $2 j >> gpurun_out/pmcw_j.txt 2>&1 || exit 1
done
cat gpurun_out/pmcw_j.txt
