#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# K3 mode-1 (k_count_scatter) ablations on one GPU's share of config 4
# (--virtual-world 8: 125M IMIX frames, 125k flows), one rocprofv3 kernel trace
# per TCBEE_K3ABL variant (timing only; outputs are wrong for variants != 0).
#   bash tools/k3_ablate.sh [variants...]     (default: 0 65 66 68 74 78 80)
set -u
mkdir -p gpurun_out/k3abl
export TMPDIR=/tmp
vs=${*:-0 65 66 68 74 78 80}
for v in $vs; do
  TCBEE_K3ABL=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/k3abl/v$v -o run \
    --output-format csv -- python bench.py --config4 --virtual-world 8 --steps 5 --warmup 1 \
    --no-cpu --no-extra --sample-check > gpurun_out/k3abl/v$v.log 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  echo "variant $v done"
done
