#!/bin/bash
# A/B session: GPU parity tests, the exhaustive probe, then tools/ab_frame.py over the given library variants
# (default + sky-only frames), each step under its own time limit.  usage: tools/ab_session.sh lib1.so lib2.so ...
set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/ab_pytest.log" 2>&1; rc=$?
tail -3 "$OUT/ab_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_frame.py --frames 30 "$@" || exit $?
timeout -k 10 200 python tools/ab_frame.py --frames 30 --cfg empty=true "$@" || exit $?
