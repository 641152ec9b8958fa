#!/bin/bash
# Two independent N=1 bench processes on the same GPU at once (no torch.distributed):
# does sharing the device between processes alone slow K1, as the gloo rehearsals
# (ranks sharing device 0) show? Then one process alone for the same size.
set -u
mkdir -p gpurun_out
A="--frames ${FRAMES:-20000000} --steps 5 --warmup 2 --no-cpu --no-extra --sample-check"
timeout -k 10 300 python bench.py $A > gpurun_out/share_p1.json 2> gpurun_out/share_p1.err &
p1=$!
timeout -k 10 300 python bench.py $A > gpurun_out/share_p2.json 2> gpurun_out/share_p2.err &
p2=$!
wait $p1; r1=$?
wait $p2; r2=$?
echo "concurrent rc $r1 $r2" >&2
[ $r1 -eq 0 ] && [ $r2 -eq 0 ] || exit 1
timeout -k 10 300 python bench.py $A > gpurun_out/share_solo.json 2> gpurun_out/share_solo.err || exit 1
for f in share_p1 share_p2 share_solo; do
  python -c "import json,sys; b=json.loads([l for l in open('gpurun_out/$f.json') if l.startswith('{')][-1]); print('$f', b['ms_per_step'], b['roofline']['k1_ms'])" >&2
done
