#!/bin/bash
# Config 2 (1M x 64 B, one flow, reset per step) under several libraries, alternating
# processes: NAMES="HEAD wt_x ..." (ab/ab_<name>/libtcbee_amd.so, tools/lib_ab.sh
# build), PAIRS rounds. Each process: tools/c2_warm.py (bench.py's own run_device).
set -u
mkdir -p gpurun_out
for r in $(seq 1 ${PAIRS:-2}); do
  for n in ${NAMES}; do
    echo "=== $n round $r"
    TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_$n/libtcbee_amd.so timeout -k 10 120 python tools/c2_warm.py --rounds 1 \
      --idle 0.5 --legs ${LEGS:-200:200,1000:1000} 2>/dev/null | tail -1 || exit $?
  done
done
