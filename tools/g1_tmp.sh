set -u
mkdir -p gpurun_out/g7
export TMPDIR=/tmp
for m in 1 4; do
timeout -k 10 300 python tools/k1_sweep.py --frames 125000000 --fpl 2 --workloads imix1M,imix10k --rounds 3 --iters 3 --flows-only --cap-mult $m --var TCBEE_WALK=0,2,8 > gpurun_out/g7/sweep_$m.log 2>&1 || { echo FAIL1; tail -20 gpurun_out/g7/sweep_$m.log; exit 1; }
echo "cap-mult $m"; grep imix gpurun_out/g7/sweep_$m.log | grep -v '^{'
done
