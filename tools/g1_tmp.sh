set -u
mkdir -p gpurun_out/g19
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29541 bench.py --steps 10 --no-cpu --no-extra > gpurun_out/g19/plain.log 2>&1 || { echo FAIL0; tail -20 gpurun_out/g19/plain.log; exit 1; }
grep '^{' gpurun_out/g19/plain.log | cut -c1-300
for ov in 0 1; do
timeout -k 10 300 env TCBEE_BENCH_FORCE_MERGE=1 TCBEE_BENCH_OVERLAP=$ov $R --master-port 2954$ov bench.py --steps 10 --no-cpu --no-extra > gpurun_out/g19/fm_$ov.log 2>&1 || { echo FAIL$ov; tail -20 gpurun_out/g19/fm_$ov.log; exit 1; }
echo "force-merge overlap=$ov"; grep '^{' gpurun_out/g19/fm_$ov.log | cut -c1-300
done
timeout -k 10 300 env TCBEE_BENCH_FORCE_MERGE=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g19/prof -o run -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --steps 5 --no-cpu --no-extra > gpurun_out/g19/prof.log 2>&1 || echo PROF_FAIL
