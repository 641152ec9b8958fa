#!/bin/bash
# One GPU-box session: parity tests, smoke, bench. Each GPU step has its own
# time limit; a crash/abort/timeout (anything but pass/fail) stops the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -25 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests)  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread ;;
    tests-all)  step pytest_gpu 900 python -m pytest tests -m gpu -q ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py ;;
    bench-short) step bench 600 python bench.py --steps 10 --cpu-seconds 6 ;;
    sweep)  step sweep 900 python tools/k1_sweep.py ;;
    sweep2) step sweep 900 python tools/k1_sweep.py --fpl 2,4 --workloads imix10k,imix1,64B1 ;;
    sweep1m) step sweep1m 900 python tools/k1_sweep.py --frames 1000000 --fpl 1,2,4 --workloads 64B1,imix10k --rounds 5 --iters 20 ;;
    pmc)    step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extra --sample-check && \
            step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extra --sample-check ;;
    dist2)  step dist2 600 env TCBEE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --frames 20000000 --steps 5 --warmup 2 ;;
    rccl1)  step rccl1 600 env TCBEE_BENCH_FORCE_MERGE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537 bench.py --config4 --steps 5 --warmup 2 --no-cpu --no-extra ;;
    dist2c4) step dist2c4 600 env TCBEE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 2 --config4 --frames 30000000 --steps 3 --warmup 1 ;;
    c4v8)   step c4v8 600 python bench.py --config4 --virtual-world 8 --steps 10 --warmup 2 --no-cpu --no-extra --sample-check ;;
    rccl1m) step rccl1m 600 env TCBEE_BENCH_FORCE_MERGE=1 TCBEE_BENCH_EXCHANGE=merge python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545 bench.py --config4 --steps 5 --warmup 2 --no-cpu --no-extra ;;
    rccl3)  step rccl3 600 env TCBEE_BENCH_FORCE_MERGE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29547 bench.py --shard flowhash --steps 20 --warmup 3 --no-cpu --no-extra --sample-check ;;
    k3range) step k3range 900 python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix20k,imix30k,imix45k,imix60k,imix125k --frames 100000000 --rounds 2 --iters 3 --var TCBEE_TEST_K3_NORANGE=0,1 ;;
    k3stage) step k3stage 900 python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix60k,imix125k,imix1M --frames 100000000 --rounds 2 --iters 3 --var TCBEE_K3ABL=0,90 ;;
    pmc3) step pmc3 1200 bash tools/pmc_c4.sh ;;
    asyncab) step asyncab0 600 env TCBEE_BENCH_ASYNC=0 python bench.py --steps 20 --no-cpu --no-extra --sample-check && \
             step asyncab1 600 env TCBEE_BENCH_ASYNC=1 python bench.py --steps 20 --no-cpu --no-extra --sample-check && \
             step asyncab2 600 env TCBEE_BENCH_ASYNC=0 python bench.py --config4 --virtual-world 8 --steps 10 --no-cpu --no-extra --sample-check && \
             step asyncab3 600 env TCBEE_BENCH_ASYNC=1 python bench.py --config4 --virtual-world 8 --steps 10 --no-cpu --no-extra --sample-check ;;
    asynccap) for g in 0 16 32 64; do step asynccap$g 600 env TCBEE_BENCH_ASYNC=1 TCBEE_ASYNC_K3_BLOCKS=$g python bench.py --steps 20 --no-cpu --no-extra --sample-check || exit 1; done; \
              for g in 0 32 64; do step asynccapc4$g 600 env TCBEE_BENCH_ASYNC=1 TCBEE_ASYNC_K3_BLOCKS=$g python bench.py --config4 --virtual-world 8 --steps 10 --no-cpu --no-extra --sample-check || exit 1; done; \
              step asynccapoff 600 env TCBEE_BENCH_ASYNC=0 python bench.py --steps 20 --no-cpu --no-extra --sample-check ;;
    capsweep) step capsweep 900 python tools/k1_sweep.py --fpl 2 --flows-only --workloads imix10k,imix125k,imix1M --frames 100000000 --rounds 2 --iters 3 --cap-mult 1,4,8,16 ;;
    smallprof) step smallprof 600 bash tools/small_prof.sh ;;
    xprof)  step xprof 600 env MASTER_ADDR=127.0.0.1 MASTER_PORT=29543 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 TCBEE_BENCH_FORCE_MERGE=1 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof -o run --output-format csv -- python bench.py --config4 --steps 5 --warmup 1 --no-cpu --no-extra --sample-check ;;
    sq)     step sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS --output-format csv -d gpurun_out/sq -o run -- python tools/k1_sweep.py --rounds 1 --iters 2 --fpl 2 --workloads imix10k ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --no-cpu --no-extra --sample-check ;;
    c4fprof) step c4fprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c4fprof -o run --output-format csv -- python bench.py --config4 --shard contig --steps 5 --warmup 1 --no-cpu --no-extra --sample-check ;;
    c4prof) step c4prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv -- python bench.py --config4 --virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra --sample-check ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
