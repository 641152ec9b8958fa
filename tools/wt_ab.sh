#!/bin/bash
# (round 6, refuted; the knob is reverted — rebuild it from the log to rerun) K1 write-through stores (TCBEE_K1_WT=16 / 18) vs the product: config 2 per step
# (tools/c2_ab.sh), K1 on config 3 and the share (tools/ab_multi.sh), the parity suite
# on the sc1 build, and a config-2 kernel trace of each for the launch gaps.
set -u
mkdir -p gpurun_out
NAMES="HEAD wt_wt16 wt_wt18" PAIRS=3 timeout -k 10 300 bash tools/c2_ab.sh > gpurun_out/wt_c2.log 2>&1 || exit 1
NAMES="wt_wt16 wt_wt18" PAIRS=2 timeout -k 10 500 bash tools/ab_multi.sh --workloads imix10k,imix125k --cap-mult 1.04 > gpurun_out/wt_k1.log 2>&1 || exit 1
for n in HEAD wt_wt16; do
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_$n/libtcbee_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wt_tr_$n -o run \
    -- python bench.py --frames 1000000 --sizes 64 --flows 1 --steps 200 --warmup 20 --no-extra --no-cpu > gpurun_out/wt_tr_$n.json 2> gpurun_out/wt_tr_$n.err || exit 1
done
TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_wt_wt16/libtcbee_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wt_parity.log 2>&1
