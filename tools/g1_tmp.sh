set -u
mkdir -p gpurun_out/g29
export TMPDIR=/tmp
timeout -k 10 600 python tools/k1_sweep.py --frames 125000000 --fpl 2 --rounds 3 --iters 3 --flows-only --var TCBEE_K3ABL=0,66,70 --workloads imix125k,imix1M,imix10k > gpurun_out/g29/sweep.log 2>&1 || { echo FAIL1; tail -20 gpurun_out/g29/sweep.log; exit 1; }
grep -E "imix" gpurun_out/g29/sweep.log | grep -v '^{'
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "k3 or merge or flowhash or over_1M" > gpurun_out/g29/pytest.log 2>&1 || { echo FAILT; tail -40 gpurun_out/g29/pytest.log; exit 1; }
tail -2 gpurun_out/g29/pytest.log
