#!/bin/bash
# Same-box A/B of the working tree's product kernels ("new") against any number of
# ab/ab_<NAME> libraries (tools/lib_ab.sh build NAME, e.g. wt:prio3 with
# HIPEXTRA=-D...): alternating processes, PAIRS rounds, tools/k1_sweep.py args.
#   NAMES="wt_prio3 wt_k3prio2" PAIRS=2 tools/ab_multi.sh --workloads imix10k,imix1M
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_multi.log
for i in $(seq 1 ${PAIRS:-2}); do
  for v in new ${NAMES:-}; do
    if [ $v = new ]; then L=""; else L="ab/ab_$v/libtcbee_amd.so"; fi
    TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$L timeout -k 10 400 python tools/k1_sweep.py --fpl 2 --flows-only "$@" \
      > gpurun_out/ab_multi_$v.log 2>&1 || { tail -5 gpurun_out/ab_multi_$v.log; exit 1; }
    grep fpl gpurun_out/ab_multi_$v.log | grep -v '^{' | sed "s/^/$v$i /" >> gpurun_out/ab_multi.log
  done
done
cat gpurun_out/ab_multi.log
