#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# A/B of K1 record-staging modes (TCBEE_STAGE) in alternating processes
for r in 1 2; do for st in 0 1; do
  echo "STAGE=$st"; TCBEE_STAGE=$st python tools/k1_sweep.py --fpl 2,4 --workloads imix10k,64B1 --rounds 2 --iters 5 2>&1 | grep -E "^(imix|64B)"
done; done
