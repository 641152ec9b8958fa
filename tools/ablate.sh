#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# Timing-only K1 ablations (TCBEE_ABLATE bits, see k_parse): one process per variant,
# two interleaved passes.
for r in 1 2; do for b in 0 1 2 4 8 16 3 31; do
  echo "ABLATE=$b"; TCBEE_ABLATE=$b python tools/k1_sweep.py --fpl 2 --workloads imix10k,64B1 --rounds 2 --iters 5 2>&1 | grep -E "^(imix|64B)"
done; done
