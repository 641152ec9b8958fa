#!/bin/bash
# Round-4 closing measurements on one box: the GPU test suite, then the headline
# trace with its bench line and the config-4 legs' traces (tools/r04_prof.sh), then
# the k_parse PMC passes of config 3, the N=8 share and the 1M-flow trace
# (tools/pmc_c4.sh). A step that times out, aborts or faults ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "=== tests rc=$rc" >&2; tail -3 gpurun_out/pytest_gpu.log >&2
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in "$@"; do
  case $s in
    prof) bash tools/r04_prof.sh prof c4 c4f || exit $? ;;
    pmc)  LEGS="${LEGS:-c3 c4v8 c4}" bash tools/pmc_c4.sh || exit $? ;;
    bench) timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err || exit $?
           tail -2 gpurun_out/bench_full.err >&2 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
