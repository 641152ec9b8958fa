set -u
mkdir -p gpurun_out/g35
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 env TCBEE_BENCH_FORCE_MERGE=1 $R --master-port 29571 bench.py --steps 10 --no-cpu --no-extra > gpurun_out/g35/fm.log 2>&1 || { echo FAILFM; tail -20 gpurun_out/g35/fm.log; exit 1; }
grep '^{' gpurun_out/g35/fm.log | cut -c1-700
timeout -k 10 600 env TCBEE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --frames 20000000 --steps 3 --warmup 1 > gpurun_out/g35/d2.log 2>&1 || { echo FAILD; tail -20 gpurun_out/g35/d2.log; exit 1; }
grep '^{' gpurun_out/g35/d2.log | cut -c1-900
