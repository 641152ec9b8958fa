#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
for r in 1 2; do for nt in 0 1; do
  echo "NT=$nt"; TCBEE_NT=$nt python tools/k1_sweep.py --fpl 2 --workloads imix10k,64B1 --rounds 2 --iters 5 2>&1 | grep -E "^(imix|64B)"
done; done
echo "small"; python tools/k1_sweep.py --frames 1000000 --fpl 2 --workloads 64B1,imix10k --rounds 3 --iters 20 2>&1 | grep -E "^(imix|64B)"
