set -u
mkdir -p gpurun_out/g21
export TMPDIR=/tmp
timeout -k 10 400 python tools/arena_alloc_ab.py > gpurun_out/g21/ab.log 2>&1 || { echo FAIL1; tail -20 gpurun_out/g21/ab.log; exit 1; }
tail -4 gpurun_out/g21/ab.log
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/g21/rd -o run -- python tools/arena_alloc_ab.py --iters 1 > gpurun_out/g21/rd.log 2>&1 || { echo FAIL2; tail -5 gpurun_out/g21/rd.log; exit 1; }
echo ok
