#!/bin/bash
# The current GPU-box session (rewritten per session; run through gpurun): every GPU step under its own time limit,
# stop at the first failure.  usage: tools/session.sh <tag> [steps...]; steps: tests smoke bench sections profile
# configs scale loops rehearse (default: tests smoke sections profile bench)
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  return $rc
}
tag=${1:-r04}; shift
steps=${*:-tests smoke sections profile bench}
for s in $steps; do
  case $s in
    tests) step pytest_$tag 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
    smoke) step smoke_$tag 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    sections) step sections_$tag 120 python tools/chain_sections.py || exit $? ;;
    profile)
      bash tools/profile_workload.sh ultracomplex_1080p64 $tag || exit $?
      step digest_$tag 60 python tools/pmc_digest.py "$OUT/prof_ultracomplex_1080p64_$tag" ultracomplex_1080p64 || exit $?
      cp profiles/pmc_ultracomplex_1080p64.json "$OUT/pmc_ultracomplex_1080p64.json" ;;
    configs)
      for w in ultracomplex_4k64 complex_4k64 ultracomplex_4k256 fsuzane_1080p64 cube_1080p16 simplest_256p1; do
        step bench_${tag}_$w 300 python bench.py --workload $w --steps 10 --warmup 3 --no-extras --no-cpu-baseline || exit $?
      done ;;
    scale)
      step scale1080_$tag 200 python tools/scale_probe.py 5 1920 1080 64 overlap || exit $?
      step scale4k_$tag 200 python tools/scale_probe.py 5 3840 2160 64 overlap || exit $?
      export SCALE_BAND=8
      step scale1080_band8_$tag 200 python tools/scale_probe.py 5 1920 1080 64 overlap || exit $?
      step scale4k_band8_$tag 200 python tools/scale_probe.py 5 3840 2160 64 overlap || exit $?
      unset SCALE_BAND ;;
    loops)
      cd /tmp
      step loop1_$tag 120 rocprofv3 --kernel-trace --stats -d "$OUT/loop1_$tag" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 40 overlap 1 || exit $?
      step loop8_$tag 120 rocprofv3 --kernel-trace --stats -d "$OUT/loop8_$tag" -o run --output-format csv -- python3 "$R/tools/frame_loop.py" 60 overlap 8 || exit $?
      cd "$R" ;;
    rehearse)
      # N > 1 rehearsal on this one GPU (explicit gloo, ranks sharing the card: the host-frame path and the small-share
      # launches, not a scaling measurement -- the 8-GPU curve is the driver's)
      for n in 2 8; do
        step rehearse${n}_$tag 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
          --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit $?
      done
      step rehearse8_band8_$tag 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29518 bench.py --gpus 8 --band 8 --backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-extras || exit $? ;;
    bench) step bench_$tag 400 python bench.py || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
