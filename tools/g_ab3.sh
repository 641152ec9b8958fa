set -u
for rev in HEAD wt:tile; do
  REV=$rev PAIRS=2 bash tools/ab_pair.sh --workloads imix10k --cap-mult 1.05 --rounds 3 --iters 5 > /dev/null 2>&1 || exit 1
  sed "s/^/[$rev] /" gpurun_out/ab_pair.log >> gpurun_out/ab3.log
  REV=$rev PAIRS=2 bash tools/ab_pair.sh --workloads 64B1 --frames 1000000 --cap-mult 1.05 --rounds 5 --iters 300 > /dev/null 2>&1 || exit 1
  sed "s/^/[$rev] /" gpurun_out/ab_pair.log >> gpurun_out/ab3.log
done
cat gpurun_out/ab3.log
