#!/bin/bash
# Round-4 A/B experiments on one box, each step under its own limit; a step that
# ends in anything but success stops the script.
#   ab:   K1 load-phase priority 3 / 1 and K3 load-phase priority 2 vs the product
#         (build/ab_* libraries, tools/lib_ab.sh build wt:NAME with HIPEXTRA)
#   k3v:  K3 mode 0 with 16-B loads of four packed words (variants build,
#         TCBEE_K3ABL=40/42) vs the product tiling (0)
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -12 "gpurun_out/$name.log" >&2
  [ $rc -eq 0 ] || exit $rc
}
for s in "$@"; do
  case $s in
    ab)  step ab 1000 env NAMES="${NAMES:-wt_prio3 wt_defer wt_k3prio2}" PAIRS=2 bash tools/ab_multi.sh \
           --workloads imix10k,imix1M,64B1 --rounds 3 --iters 5 ;;
    k3v) step k3v 400 python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix10k,64B1 \
           --var TCBEE_K3ABL=0,40,42 --rounds 3 --iters 5 ;;
    c2ab) step c2ab 600 env NAMES="${NAMES:-HEAD~1}" PAIRS=3 bash tools/ab_multi.sh \
           --frames 1000000 --workloads 64B1,imix10k --rounds 5 --iters 20 --min-table 64 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
             > gpurun_out/pytest_gpu.log 2>&1
           rc=$?; echo "=== tests rc=$rc" >&2; tail -5 gpurun_out/pytest_gpu.log >&2
           [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    dist) step dist 900 bash tools/dist_rehearsal.sh n2 n8 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
