#!/bin/bash
# Flow-table load factor A/B (round 3 compact table): max_flows = mult x flows
# (slots = 2 x max_flows), 125M IMIX frames, 10k / 125k / 1M flows, one process,
# under a kernel trace (K1 and K3 durations per variant).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/capab -o run --output-format csv \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads ${WL:-imix10k,imix125k,imix1M} \
  --frames 125000000 --rounds 2 --iters 3 --cap-mult ${MULTS:-1,4,8} \
  > gpurun_out/capab.log 2>&1
rc=$?
echo "=== capab rc=$rc" >&2
grep -v "^W20\|^E20" gpurun_out/capab.log | tail -12 >&2
exit $rc
