#!/bin/bash
# run pytest selections one after another; continue past test failures (rc 1), stop on anything else
mkdir -p gpurun_out
i=0
for sel in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$sel" > gpurun_out/bis_$i.log 2>&1
  rc=$?
  echo "sel $i [$sel] rc=$rc $(tail -n 1 gpurun_out/bis_$i.log)" | tee -a gpurun_out/bis_summary.log
  [ $rc -le 1 ] || exit $rc
done
