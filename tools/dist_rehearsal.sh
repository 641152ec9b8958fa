#!/bin/bash
# N>1 rehearsal of the driver's scaling command on a one-GPU box: the ranks share
# device 0 over gloo (RCCL refuses two ranks on one GPU). Each step has its own
# time limit; the first failure ends the script.
set -u
mkdir -p gpurun_out
run() {  # name timeout nproc args...
  local name=$1 to=$2 np=$3; shift 3
  echo "=== $name" >&2
  TCBEE_DIST_BACKEND=gloo timeout -k 10 "$to" python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$np" --master-addr 127.0.0.1 --master-port $((29600 + np)) \
    bench.py --gpus "$np" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.err" >&2
  cat "gpurun_out/$name.json" >&2
  [ $rc -eq 0 ] || exit $rc
}
for s in "$@"; do
  case $s in
    n2)   run dist_n2 600 2 --steps 5 --warmup 2 --c4-frames 40000000 ;;
    n2full) run dist_n2full 900 2 ;;  # the driver's own N=2 command, default sizes
    n4)   run dist_n4 600 4 --frames 20000000 --steps 5 --warmup 2 --c4-frames 16000000 ;;
    n8)   run dist_n8 600 8 --frames 8000000 --steps 5 --warmup 2 --c4-frames 6000000 ;;
    n2c4) run dist_n2c4 600 2 --config4 --frames 40000000 --steps 3 --warmup 1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
