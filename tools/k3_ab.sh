#!/bin/bash
export TCBEE_AB_LIB=${TCBEE_AB_LIB:-tcbee_amd/lib/libtcbee_amd_variants.so}  # TCBEE_* variants: variants build only
# K3 mode-1 A/B (round 3): k_count_chunk2 (default, 12288-record chunks, two
# workgroups per CU; 94 = its 512-thread form) vs round 2's k_count_chunk (93), on
# the config-4 share's flow count (125k) and the whole 1M-flow trace, 125M frames,
# under a kernel trace (per-kernel durations of every variant in one process).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/k3ab -o run --output-format csv \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads ${WL:-imix125k,imix1M} \
  --frames 125000000 --rounds 2 --iters 3 --var TCBEE_K3ABL=${VARS:-0,93,94} \
  > gpurun_out/k3ab.log 2>&1
rc=$?
echo "=== k3ab rc=$rc" >&2
tail -30 gpurun_out/k3ab.log >&2
exit $rc
