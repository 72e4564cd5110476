#!/bin/bash
# One BASELINE workload (bench.py --workload) under each given library, three times (not part of the product).
# usage: tools/cfg_ab.sh <tag> <workload> lib1.so lib2.so ...
set -u
tag=$1; w=$2; shift 2
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
for rep in 1 2 3; do
  for l in "$@"; do
    RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l timeout -k 10 200 python bench.py --workload "$w" --steps 10 --warmup 3 \
      --no-extras --no-cpu-baseline > "$OUT/cfg_ab.log" 2>&1 || { echo "$l failed"; tail -5 "$OUT/cfg_ab.log"; exit 1; }
    python3 - "$l" "$rep" "$w" >> "$OUT/cfg_ab_$tag.log" <<'P'
import json, sys
d = json.loads([l for l in open("gpurun_out/cfg_ab.log") if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f"rep {sys.argv[2]} {sys.argv[1]:24s} {sys.argv[3]} frame {d['ms_per_step']:.4f} chain {k['rtc_render_chain']['ms']:.4f} "
      f"sky {k['rtc_render_sky']['ms']:.4f} equal {d['host_frame_equals_rtc_render']}")
P
  done
done
cat "$OUT/cfg_ab_$tag.log"
