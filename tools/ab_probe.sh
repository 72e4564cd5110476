#!/bin/bash
# A/B timing of library variants: tools/ab_probe.sh lib1 lib2 ...  (each under raytracingc_amd/_lib/)
mkdir -p gpurun_out
for l in "$@"; do
  echo "== $l"
  RTC_LIB_PATH=$PWD/raytracingc_amd/_lib/$l timeout -k 10 240 python tools/kernel_probe.py ${PROBE_ARGS:-} || exit $?
done
