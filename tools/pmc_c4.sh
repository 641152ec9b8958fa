#!/bin/bash
# HBM traffic (separate --pmc passes, MI355X_MICROARCH.md "HBM") of the config-4
# legs: the whole 1M-flow trace on one GPU (--config4) and one GPU's flow-hash
# share at N=8 (--config4 --virtual-world 8), plus the config-3 headline. Each
# pass is its own short run under a hard time limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name counters... -- bench args
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done
  shift
  timeout -s KILL 300 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d "gpurun_out/$name" -o run \
    -- python bench.py --steps 2 --warmup 1 --no-cpu --no-extra --sample-check "$@" \
    > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
for leg in ${LEGS:-c3 c4 c4v8 v6}; do
  case $leg in
    v6) args=(--sizes imix6) ;;
    c2) args=(--frames 1000000 --sizes 64 --flows 1) ;;
    c3) args=() ;;
    c4) args=(--config4) ;;
    c4v8) args=(--config4 --virtual-world 8) ;;
  esac
  run "pmc_${leg}_fetch" FETCH_SIZE -- "${args[@]}"
  run "pmc_${leg}_write" WRITE_SIZE -- "${args[@]}"
  run "pmc_${leg}_rdreq" TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum -- "${args[@]}"
done
