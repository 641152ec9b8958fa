#!/bin/bash
# (round 6, refuted and reverted: profiles/r06_rank_count_ab.log; the knob TCBEE_RANK_COUNT no longer exists)
# K2 as one counting launch (k_rank_count, the product) vs the bitmap path
# (ab/ab_wt_rk0: tools/lib_ab.sh build wt:rk0 with HIPEXTRA=-DTCBEE_RANK_COUNT=0):
# the GPU suite on the product, then config 3 alternating processes, then the
# headline under the kernel trace for the per-launch gaps.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${RK_TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rk_pytest.log 2>&1 || { tail -30 gpurun_out/rk_pytest.log; exit 1; }
tail -2 gpurun_out/rk_pytest.log
for i in 1 2 3 4; do for n in new wt_rk0; do
  if [ $n = new ]; then L=""; else L=ab/ab_$n/libtcbee_amd.so; fi
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=$L timeout -k 10 200 python bench.py --no-extra --no-cpu > gpurun_out/rk_${n}_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/rk_${n}_$i.json').read().strip().splitlines()[-1]);print('$n',d['value'],d['ms_per_step'],d['roofline']['k1_ms'],d['check']['full_bit_exact'])"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rk_tr -o run -- python bench.py --no-extra --no-cpu > gpurun_out/rk_tr.json 2>/dev/null
TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_wt_rk0/libtcbee_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rk0_tr -o run -- python bench.py --no-extra --no-cpu > gpurun_out/rk0_tr.json 2>/dev/null
