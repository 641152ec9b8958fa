#!/bin/bash
# K1 timing-event flags A/B (round 6, profiles/r06_prof_event_ab.log): config 2 per step
# (tools/c2_ab.sh) and config 3 for three builds, then a kernel trace of the kept one.
# Build first, here: HIPEXTRA=-DTCBEE_PROF_EVFLAGS=0 tools/lib_ab.sh build wt:evdef;
# HIPEXTRA=-DTCBEE_PROF_EVFLAGS=hipEventReleaseToDevice tools/lib_ab.sh build wt:evdev;
# tools/lib_ab.sh build wt:evnf (the default, hipEventDisableSystemFence).
set -u
mkdir -p gpurun_out
NAMES="wt_evdef wt_evnf wt_evdev" PAIRS=3 timeout -k 10 300 bash tools/c2_ab.sh > gpurun_out/ev_c2.log 2>&1 || exit 1
for i in 1 2; do for n in wt_evdef wt_evnf; do
  TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_$n/libtcbee_amd.so timeout -k 10 200 python bench.py --no-extra --no-cpu > gpurun_out/ev_c3_${n}_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ev_c3_${n}_$i.json').read().strip().splitlines()[-1]);print('$n',d['value'],d['ms_per_step'],d['roofline']['k1_ms'])"
done; done
TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_wt_evnf/libtcbee_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_tr -o run -- python bench.py --no-extra --no-cpu > gpurun_out/ev_tr.json 2>/dev/null
