#!/bin/bash
# K1 under a second process's kernels on the same GPU: world-2 gloo flow-hash runs
# (both ranks on device 0, their K1s launched at the same moments) vs one process,
# for the working tree's library and each ab/ab_<NAME> given in NAMES.
set -u
mkdir -p gpurun_out
F=${FRAMES:-10000000}
A="--frames $F --steps ${STEPS:-30} --warmup 3 --no-cpu --no-extra --sample-check"
one() {  # tag lib
  local tag=$1 lib=$2
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$lib timeout -k 10 300 python bench.py $A > gpurun_out/lbc_${tag}_solo.json 2> gpurun_out/lbc_${tag}_solo.err || exit 1
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$lib TCBEE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 $A \
    > gpurun_out/lbc_${tag}_n2.json 2> gpurun_out/lbc_${tag}_n2.err || exit 1
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$lib timeout -k 10 200 python tools/k1_concurrent.py --frames $F >&2 || exit 1
  for m in solo n2; do
    python -c "import json; b=json.loads([l for l in open('gpurun_out/lbc_${tag}_$m.json') if l.startswith('{')][-1]); print('$tag $m', 'step', b['ms_per_step'], 'K1', b['roofline']['k1_ms'])" >&2
  done
}
python -c "
import ctypes as C
h = C.CDLL('libamdhip64.so'); v = C.c_int()
h.hipDeviceGetAttribute(C.byref(v), 10017, 0)  # hipDeviceAttributeWallClockRate (kHz)
print('wall clock kHz', v.value)" >&2
one wt tcbee_amd/lib/libtcbee_amd.so
for n in ${NAMES:-}; do one $n ab/ab_$n/libtcbee_amd.so; done
