set -u
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g8/pytest.log 2>&1 || { echo FAILT; tail -40 gpurun_out/g8/pytest.log; exit 1; }
tail -2 gpurun_out/g8/pytest.log
timeout -k 10 300 python tools/k1_sweep.py --frames 100000000 --fpl 2 --workloads imix10k,imix1 --rounds 3 --iters 5 --flows-only --var TCBEE_TEST_NOPACK=0,1 > gpurun_out/g8/sweep.log 2>&1 || { echo FAIL1; tail -20 gpurun_out/g8/sweep.log; exit 1; }
grep imix gpurun_out/g8/sweep.log | grep -v '^{'
