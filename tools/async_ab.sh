#!/bin/bash
# K3 on a side stream beside the next step's K1 (TCBEE_BENCH_ASYNC=1) vs in line, config 3,
# alternating processes (round 6, profiles/r06_async_ids_ab.log).
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for a in 0 1; do
    TCBEE_BENCH_ASYNC=$a timeout -k 10 200 python bench.py --no-extra --no-cpu > gpurun_out/async_${a}_$i.json 2> gpurun_out/async_${a}_$i.err || exit 1
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/async_${a}_$i.json').read().strip().splitlines()[-1]);print('async=$a run $i',d['value'],d['ms_per_step'],d['roofline']['k1_ms'],d['check']['full_bit_exact'])"
  done
done
