#!/bin/bash
# rocprofv3 counter passes (one pass per --pmc group; no tracing domains besides kernel-trace)
# usage: tools/pmc.sh <variant> <name> <counters...>
set -u
R=$(pwd); V=$1; N=$2; shift 2
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$R/gpurun_out/$N" -o p --output-format csv -- python3 "$R/tools/one_render.py" "$V" > "$R/gpurun_out/$N.log" 2>&1
rc=$?; echo "$N rc=$rc"; exit $rc
