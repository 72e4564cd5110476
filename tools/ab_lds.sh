#!/bin/bash
# LDS counters of the timed rtc_render_chain launch per library variant: tools/ab_lds.sh lib1.so lib2.so ...
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
G4="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAVES"
for l in "$@"; do
  export RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G4 -d "$R/gpurun_out/lds_$l" -o p --output-format csv \
    -- python3 "$R/tools/one_render.py" ultracomplex_1080p64 1 > "$R/gpurun_out/lds_$l.log" 2>&1) || { echo "$l pmc failed"; exit 1; }
  python3 - "$R/gpurun_out/lds_$l" "$l" <<'P'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f)):
    if "rtc_render_chain<false, false>" in row["Kernel_Name"]:
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
print(sys.argv[2], {k: int(v) for k, v in sorted(acc.items())})
P
done
