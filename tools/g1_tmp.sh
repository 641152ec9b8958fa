set -u
mkdir -p gpurun_out/g34
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 300 env PF_LIST=0,8,32,64 python tools/e2e_ab.py . >> gpurun_out/g34/e2e.log 2>&1 || { echo FAIL; tail -20 gpurun_out/g34/e2e.log; exit 1; }
done
grep Mpkt gpurun_out/g34/e2e.log
