#!/bin/bash
# Rank-share A/B over library variants: tools/ab_scale.sh kernel lib1.so lib2.so ...
# (SCALE_NS selects the N; every share of each N on this one GPU, tools/scale_probe.py)
set -u
kernel=$1; shift
for l in "$@"; do
  RTC_LIB_PATH=$GRAFT_REPO_ROOT/raytracingc_amd/_lib/$l timeout -k 10 240 python tools/scale_probe.py 5 1920 1080 64 $kernel \
    > gpurun_out/abs.log 2>&1 || { echo "$l failed"; tail -5 gpurun_out/abs.log; exit 1; }
  sed "s/^/$l $kernel /" gpurun_out/abs.log | grep '"n"'
done
