set -u
mkdir -p gpurun_out/g25
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/g25/pytest.log 2>&1 || { echo FAILT; tail -40 gpurun_out/g25/pytest.log; exit 1; }
tail -2 gpurun_out/g25/pytest.log
timeout -k 10 600 python -u bench.py --config4 --steps 5 --warmup 1 --no-cpu > gpurun_out/g25/c4.log 2>&1 || { echo FAILC4; tail -20 gpurun_out/g25/c4.log; exit 1; }
grep '^{' gpurun_out/g25/c4.log | cut -c1-900
timeout -k 10 600 env TCBEE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --shard flowhash --frames 10000000 --flows 100000 --steps 3 --warmup 1 > gpurun_out/g25/fh2.log 2>&1 || { echo FAILD; tail -20 gpurun_out/g25/fh2.log; exit 1; }
grep '^{' gpurun_out/g25/fh2.log | cut -c1-900
