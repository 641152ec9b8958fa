set -u
mkdir -p gpurun_out/g14
export TMPDIR=/tmp
W="python tools/k1_sweep.py --frames 100000000 --fpl 2 --workloads imix10k,64B1 --rounds 1 --iters 1 --flows-only"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/g14/p1 -o run -- $W > gpurun_out/g14/p1.log 2>&1 || { echo FAIL1; tail -5 gpurun_out/g14/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/g14/p2 -o run -- $W > gpurun_out/g14/p2.log 2>&1 || { echo FAIL2; tail -5 gpurun_out/g14/p2.log; exit 1; }
echo ok
