#!/bin/bash
# Per-round profiles (one box; TAG names the round, default r06): the headline command
# under rocprofv3 --kernel-trace --stats WITH the bench line that same process prints
# (the line's event-timed K1 and the trace's k_parse average come from one run), the
# config-2 / IPv6 legs, the config-4 legs' traces — one GPU's flow-hash share at N=8
# and the whole 1M-flow trace — and the K1 PMC passes (tools/pmc_c4.sh, LEGS). A
# failing step ends the script.
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
  c3)   prof ${TAG:-r06}prof_c3 400 -- --no-extra --no-cpu ;;
  c4v8) prof ${TAG:-r06}prof_c4v8 400 -- --config4 --virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra ;;
  c4)   prof ${TAG:-r06}prof_c4 400 -- --config4 --shard contig --steps 5 --warmup 1 --no-cpu --no-extra ;;
  c2)   prof ${TAG:-r06}prof_c2 300 -- --frames 1000000 --sizes 64 --flows 1 --no-extra --no-cpu --steps 200 --warmup 20 ;;
  v6)   prof ${TAG:-r06}prof_v6 400 -- --sizes imix6 --no-extra --no-cpu ;;
  pmc)  LEGS="${LEGS:-c3 c4v8}" bash tools/pmc_c4.sh || exit $? ;;
esac; done
