#!/bin/bash
# Correctness under contention: two independent bench processes on the same GPU at
# once (their steps overlap, so K1's look-back recounts and publishes predecessors),
# each checking its last step's records, ids and table in full against the oracle.
set -u
mkdir -p gpurun_out
A="--frames ${FRAMES:-20000000} --steps ${STEPS:-60} --warmup 2 --no-cpu --no-extra"
for i in 1 2; do
  timeout -k 10 400 python bench.py $A > gpurun_out/cc_$i.json 2> gpurun_out/cc_$i.err &
  eval p$i=$!
done
wait $p1; r1=$?; wait $p2; r2=$?
for i in 1 2; do
  python -c "import json; b=json.loads([l for l in open('gpurun_out/cc_$i.json') if l.startswith('{')][-1]); c=b['check']; print('process $i: K1', b['roofline']['k1_ms'], 'ms, full_bit_exact', c['full_bit_exact'], 'table', c['flow_table_exact'], 'status', c['status'])" >&2
done
[ $r1 -eq 0 ] && [ $r2 -eq 0 ]
