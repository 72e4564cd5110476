#!/bin/bash
# 1080p N = 4 / 8 shares (tools/scale_probe.py overlap) under each given library, twice, each run under its own limit
# (not part of the product).  usage: tools/scale_ab.sh <tag> lib1.so lib2.so ...
set -u
tag=$1; shift
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
for rep in 1 2; do
  for l in "$@"; do
    RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l SCALE_NS=4,8 timeout -k 10 200 python tools/scale_probe.py 5 1920 1080 64 overlap \
      > "$OUT/sab.log" 2>&1 || { echo "$l failed"; tail -5 "$OUT/sab.log"; exit 1; }
    python3 - "$l" "$rep" >> "$OUT/scale_ab_$tag.log" <<'P'
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/sab.log") if l.startswith("{")]
print(f"rep {sys.argv[2]} {sys.argv[1]:24s} " + " ".join(f"N={r['n']} slowest {r['slowest_ms']:.4f}" for r in rows))
P
  done
done
cat "$OUT/scale_ab_$tag.log"
