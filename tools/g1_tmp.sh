set -u
mkdir -p gpurun_out/g23
export TMPDIR=/tmp
for r in tmp_old . tmp_old .; do
timeout -k 10 300 python tools/e2e_ab.py $r >> gpurun_out/g23/e2e.log 2>&1 || { echo FAIL; tail -20 gpurun_out/g23/e2e.log; exit 1; }
done
grep Mpkt gpurun_out/g23/e2e.log
