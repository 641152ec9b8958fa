#!/bin/bash
# Round-5 first measurements (one box): (1) the ceiling of an L2-sized first-level
# probe — K1 with every IPv4 probe inside a 16 MiB / 4 MiB / 2 MiB / 512 KiB window
# (variants TCBEE_ABLATE=96/352/224/480) at 10k / 125k / 1M flows; (2) the L2->fabric
# read requests of the 2 MiB window at 125k flows; (3) where k_count_chunk2's time
# goes (TCBEE_K3ABL=101..107, kernel trace); (4) config 2 against round 3's kernels.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc" >&2; [ $rc -eq 0 ] || { tail -5 gpurun_out/$name.log >&2; exit $rc; }; }
case ${1:-all} in all|ceil)
step ceil 400 python -u tools/k1_sweep.py --fpl 2 --flows-only --workloads imix125k,imix1M,imix10k \
  --var TCBEE_ABLATE=0,96,352,224,480 --rounds 3 --iters 5
grep fpl gpurun_out/ceil.log | grep -v '^{' >&2 ;; esac
case ${1:-all} in all|rdreq)
step rdreq 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/rdreq -o run \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix125k --var TCBEE_ABLATE=0,224,480 --rounds 1 --iters 2 ;; esac
case ${1:-all} in all|k3)
step k3abl 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k3abl -o run \
  -- python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix1M,imix125k --var TCBEE_K3ABL=0,101,102,104,107 --rounds 2 --iters 5
grep fpl gpurun_out/k3abl.log | grep -v '^{' >&2 ;; esac
case ${1:-all} in all|c2)
NAMES="e2930e7 HEAD" PAIRS=3 LEGS=1000:1000 step c2ab 400 bash tools/c2_ab.sh
cat gpurun_out/c2ab.log >&2 ;; esac
