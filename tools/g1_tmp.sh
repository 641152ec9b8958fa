set -u
mkdir -p gpurun_out/g24
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/g24/bench.log 2>&1 || { echo FAILB; tail -30 gpurun_out/g24/bench.log; exit 1; }
tail -1 gpurun_out/g24/bench.log
