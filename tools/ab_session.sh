#!/bin/bash
# A/B of library variants on the GPU box (not part of the product): for each repetition and each library, the headline
# frame (bench.py, pipelined, D2H included; chain / sky kernel times), the slowest 1080p 1/8 and 1/4 shares
# (tools/scale_probe.py overlap) and, with AB_FSUZANE=1, C3 fsuzane.  Every step under its own time limit; stops at the
# first failure.  usage: tools/ab_session.sh <tag> lib1.so lib2.so ...   (libraries under raytracingc_amd/_lib/)
set -u
export TMPDIR=/tmp
tag=$1; shift
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
SUM=$OUT/ab_$tag.log
: > "$SUM"
for rep in $(seq 1 ${AB_REPS:-2}); do
  for l in "$@"; do
    export RTC_LIB_PATH=$R/raytracingc_amd/_lib/$l
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/ab_bench.log" 2>&1 ||
      { echo "$l bench failed" | tee -a "$SUM"; tail -20 "$OUT/ab_bench.log"; exit 1; }
    python3 - "$l" "$rep" >> "$SUM" <<'P'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab_bench.log") if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f"rep {sys.argv[2]} {sys.argv[1]:24s} frame {d['ms_per_step']:.4f} chain {k['rtc_render_chain']['ms']:.4f} "
      f"sky {k['rtc_render_sky']['ms']:.4f} moving {d['moving_camera']['ms_per_step']:.4f} equal {d['host_frame_equals_rtc_render']}")
P
    SCALE_NS=4,8 timeout -k 10 200 python tools/scale_probe.py 5 1920 1080 64 overlap > "$OUT/ab_scale.log" 2>&1 ||
      { echo "$l scale failed" | tee -a "$SUM"; tail -20 "$OUT/ab_scale.log"; exit 1; }
    python3 - "$l" "$rep" >> "$SUM" <<'P'
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/ab_scale.log") if l.startswith("{")]
print(f"rep {sys.argv[2]} {sys.argv[1]:24s} " + " ".join(f"N={r['n']} slowest {r['slowest_ms']:.4f}" for r in rows))
P
    if [ "${AB_FSUZANE:-0}" = 1 ]; then
      timeout -k 10 200 python bench.py --workload fsuzane_1080p64 --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
        > "$OUT/ab_fs.log" 2>&1 || { echo "$l fsuzane failed" | tee -a "$SUM"; exit 1; }
      python3 - "$l" "$rep" >> "$SUM" <<'P'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab_fs.log") if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f"rep {sys.argv[2]} {sys.argv[1]:24s} fsuzane frame {d['ms_per_step']:.4f} chain {k['rtc_render_chain']['ms']:.4f} "
      f"equal {d['host_frame_equals_rtc_render']}")
P
    fi
  done
done
cat "$SUM"
