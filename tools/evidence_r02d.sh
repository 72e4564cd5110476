#!/bin/bash
# Round-2 evidence session: rocprofv3 kernel-trace + PMC passes (tools/prof_session.sh), the rank-share scale
# probes (1080p x64, 4K x64) and a device-only kernel trace of back-to-back frames.  Every GPU step has its own
# time limit; the script stops at the first failing step.  usage: tools/evidence_r02d.sh [tag]
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out; tag=${1:-r02_d}
mkdir -p "$OUT"
bash tools/prof_session.sh "$tag" || exit $?
cd "$R"
timeout -k 10 200 python tools/scale_probe.py 7 > "$OUT/scale_1080_$tag.log" 2>&1 || exit $?
timeout -k 10 200 python tools/scale_probe.py 5 3840 2160 64 > "$OUT/scale_4k_$tag.log" 2>&1 || exit $?
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/loop_$tag" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 > "$OUT/loop_$tag.log" 2>&1 || exit $?
echo done
