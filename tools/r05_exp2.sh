#!/bin/bash
# Round 5: the L2-sized first-level probe ceiling, measured right (the variants
# build reads TCBEE_ABLATE per launch: k1_sweep now sets it per variant), with the
# bench's table sizing (max_flows = 1.04 x flows) at 125k / 1M flows and round 3's
# 4x sizing at 1M; then k_count_chunk2's ablations at 1M flows with packed words.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc" >&2; [ $rc -eq 0 ] || { tail -5 gpurun_out/$name.log >&2; exit $rc; }; }
step ceil2 400 python -u tools/k1_sweep.py --fpl 2 --flows-only --workloads imix125k,imix1M,imix10k \
  --var TCBEE_ABLATE=0,96,352,224,480 --rounds 3 --iters 5 --cap-mult 1.04
grep fpl gpurun_out/ceil2.log | grep -v '^{' >&2
step ceil4x 300 python -u tools/k1_sweep.py --fpl 2 --flows-only --workloads imix1M \
  --var TCBEE_ABLATE=0,96,352,224,480 --rounds 3 --iters 5
grep fpl gpurun_out/ceil4x.log | grep -v '^{' >&2
step rdreq2 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/rdreq2 -o run \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix125k --var TCBEE_ABLATE=0,96,352,224,480 --rounds 1 --iters 2 --cap-mult 1.04
step k3abl2 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k3abl2 -o run \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix1M,imix125k --var TCBEE_K3ABL=0,101,102,104,107 --rounds 2 --iters 5 --cap-mult 1.04
grep fpl gpurun_out/k3abl2.log | grep -v '^{' >&2
