#!/bin/bash
# Build an experimental librtc variant: tools/build_variant.sh <name> [extra hipcc flags...]
# -> raytracingc_amd/_lib/librtc_<name>.so  (for tools/ab_frame.py; never the product)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p /tmp/rtc_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -fPIC -std=c++17 "$@" \
  -c raytracingc_amd/csrc/rtc_render.hip -o /tmp/rtc_variants/$name.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A14 "Function Name: _Z16rtc_render_chain" | grep -E "VGPRs:|Spill|Occupancy|Scratch" \
  | sed "s/.*remark: *//;s/ \[.*//" | tr '\n' ' '; echo "<- $name"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/rtc_variants/$name.o build/rtc_frame.o build/rtc_scene.o build/rtc_probe.o build/rtc_plan.o build/scene_build.o \
  -o raytracingc_amd/_lib/librtc_$name.so -ldl -L/opt/rocm/lib -lhsa-runtime64
