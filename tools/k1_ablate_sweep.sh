#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# K1 cost breakdown (timing-only ablations, TCBEE_ABLATE bits of k_parse: 1 no
# look-back, 2 no record stores, 4 no header loads, 8 no index loads, 16 no side
# outputs): one process per setting (the launcher reads the variable once), same
# box, config-3 workload (100M IMIX frames, 10k flows), flows on and off.
set -u
mkdir -p gpurun_out
: > gpurun_out/k1_ablate.log
for a in ${ABLS:-0 1 2 4 8 16 3 31}; do
  TCBEE_ABLATE=$a timeout -k 10 120 python tools/k1_sweep.py --fpl 2 --workloads ${WL:-imix10k} \
    --rounds 3 --iters 5 > gpurun_out/k1_abl_$a.log 2>&1 || exit $?
  grep fpl gpurun_out/k1_abl_$a.log | grep -v '^{' | sed "s/^/ABL=$a /" >> gpurun_out/k1_ablate.log
done
cat gpurun_out/k1_ablate.log
