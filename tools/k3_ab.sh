#!/bin/bash
# K3 mode-1 A/B on one box: the working tree's product library ("new") against
# ab/ab_<NAME> libraries (tools/lib_ab.sh build wt:NAME with HIPEXTRA=-D...),
# alternating processes, each under rocprofv3 --kernel-trace (per-kernel times by
# template name); 125k / 1M flows, max_flows = 1.04 x flows (bench.py sizing).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 ${PAIRS:-2}); do
  for v in new ${NAMES}; do
    if [ $v = new ]; then L=tcbee_amd/lib/libtcbee_amd.so; else L=ab/ab_$v/libtcbee_amd.so; fi
    TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k3ab_${v}_$i -o run \
      -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads ${WL:-imix125k,imix1M} --cap-mult 1.04 --rounds 2 --iters 5 \
      > gpurun_out/k3ab_${v}_$i.log 2>&1 || { echo "=== $v $i failed"; tail -5 gpurun_out/k3ab_${v}_$i.log; exit 1; }
    grep fpl gpurun_out/k3ab_${v}_$i.log | grep -v '^{' | sed "s/^/$v$i /"
  done
done
