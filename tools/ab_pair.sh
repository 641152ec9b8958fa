#!/bin/bash
# Same-box A/B of the working tree's kernels (new) against build/ab_<REV> (old,
# tools/lib_ab.sh build REV): alternating processes, PAIRS times, k1_sweep args.
#   REV=HEAD PAIRS=2 tools/ab_pair.sh --workloads 64B1 --frames 1000000 ...
set -u
mkdir -p gpurun_out
rev=${REV:-HEAD}
: > gpurun_out/ab_pair.log
for i in $(seq 1 ${PAIRS:-2}); do
  for v in new old; do
    if [ $v = new ]; then L=""; else L="build/ab_${rev//:/_}/libtcbee_amd.so"; fi
    TCBEE_AB_LIB=$L timeout -k 10 300 python tools/k1_sweep.py --fpl 2 --flows-only "$@" \
      > gpurun_out/ab_pair_$v.log 2>&1 || { tail -5 gpurun_out/ab_pair_$v.log; exit 1; }
    grep fpl gpurun_out/ab_pair_$v.log | grep -v '^{' | sed "s/^/$v$i /" >> gpurun_out/ab_pair.log
  done
done
cat gpurun_out/ab_pair.log
