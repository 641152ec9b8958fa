#!/bin/bash
# Round-5 profiles (one box): the headline command under rocprofv3 --kernel-trace
# --stats WITH the bench line that same process prints (the line's event-timed K1 and
# the trace's k_parse average come from one run), then the config-4 legs' traces —
# one GPU's flow-hash share at N=8 and the whole 1M-flow trace — and the K1 PMC passes
# of config 3 and the share (tools/pmc_c4.sh). A failing step ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
prof() {  # name limit -- bench args
  local name=$1 t=$2; shift 3
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run \
    -- python bench.py "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err
  local rc=$?; echo "=== $name rc=$rc" >&2; [ $rc -eq 0 ] || { tail -5 gpurun_out/$name.err >&2; exit $rc; }
}
for s in "$@"; do case $s in
  c3)   prof r05prof_c3 400 -- --no-extra --no-cpu ;;
  c4v8) prof r05prof_c4v8 400 -- --config4 --virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra ;;
  c4)   prof r05prof_c4 400 -- --config4 --shard contig --steps 5 --warmup 1 --no-cpu --no-extra ;;
  pmc)  LEGS="${LEGS:-c3 c4v8}" bash tools/pmc_c4.sh || exit $? ;;
esac; done
