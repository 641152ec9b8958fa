#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# K1 variant A/B (TCBEE_K1V), one process, interleaved rounds (tools/k1_sweep.py).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python tools/k1_sweep.py --fpl 2 --flows-only --workloads ${WL:-imix10k,imix125k,imix1M} \
  --frames ${FRAMES:-100000000} --rounds ${ROUNDS:-3} --iters 5 --var TCBEE_K1V=${VARS:-0,30} \
  > gpurun_out/k1v.log 2>&1
rc=$?
echo "=== k1v rc=$rc" >&2
grep -v "^W20\|^E20\|^{" gpurun_out/k1v.log | tail -12 >&2
exit $rc
