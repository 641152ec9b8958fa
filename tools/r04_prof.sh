#!/bin/bash
# Round-4 profiles: the rocprofv3 kernel trace of the headline
# command WITH the bench line that same process printed (so the line's roofline
# frac and the trace's k_parse average come from one run), then the k_parse
# FETCH/WRITE/RDREQ PMC passes of config 3, the config-4 share of N=8 and the whole
# 1M-flow trace (tools/pmc_c4.sh), and kernel traces of both config-4 legs.
# Each GPU step has its own time limit; the first failure ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -4 "gpurun_out/$name.log" >&2
  [ $rc -eq 0 ] || exit $rc
}
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(prof c4 c4f)
for s in "${steps[@]}"; do
  case $s in
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
            -- python bench.py --steps 10 --no-cpu --no-extra --sample-check
          grep '^{' gpurun_out/prof.log > gpurun_out/bench.log ;;
    pmc)  step pmc 1100 env LEGS="${LEGS:-c3 c4v8 c4}" bash tools/pmc_c4.sh ;;
    c4)   step c4prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv \
            -- python bench.py --config4 --virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra --sample-check ;;
    c4f)  step c4fprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c4fprof -o run --output-format csv \
            -- python bench.py --config4 --shard contig --steps 5 --warmup 1 --no-cpu --no-extra --sample-check ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
