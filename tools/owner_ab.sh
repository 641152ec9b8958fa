set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 180 --timeout-method thread -k "owner" > gpurun_out/owner_tests.log 2>&1 || exit 1
for ex in merge owner; do
  TCBEE_BENCH_EXCHANGE=$ex TCBEE_BENCH_FORCE_MERGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$((RANDOM%9)) bench.py --config4 --shard contig --steps 5 --warmup 2 --no-cpu --no-extra --sample-check > gpurun_out/owner_$ex.log 2>&1 || exit 1
done
