#!/bin/bash
# The GPU test suite on the current tree (all of it, or one file: tests-<name>), the
# smoke, then a same-box A/B of the product K1/K3 against ab/ab_<NAME>
# (tools/lib_ab.sh build) on config 3 and the 125k-flow share shape. Each step under
# its own limit; a failure stops the script.
#   bash tools/gpu_check.sh tests smoke ab
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc" >&2; tail -4 gpurun_out/$name.log >&2; [ $rc -eq 0 ] || exit $rc; }
for s in "$@"; do case $s in
  tests) step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
  tests-*) step pytest_${s#tests-} 1000 python -u -m pytest tests/test_${s#tests-}.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
  ab) NAMES=${NAMES:-HEAD} PAIRS=${PAIRS:-2} step ab 900 bash tools/ab_multi.sh --workloads imix10k,imix125k --cap-mult 1.04 ;;
  smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
esac; done
