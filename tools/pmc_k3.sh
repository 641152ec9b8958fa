#!/bin/bash
# K3 mode 1 on one GPU's flow-hash share of config 4 (--config4 --virtual-world 8:
# ~125M IMIX frames, ~125k flows): kernel trace, then FETCH_SIZE and WRITE_SIZE
# in passes of their own (MI355X_MICROARCH.md "HBM"). Each run under a hard limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
args=(--config4 --virtual-world 8 --no-cpu --no-extra --sample-check)
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k3prof -o run \
  -- python bench.py --steps 5 --warmup 1 "${args[@]}" > gpurun_out/k3prof.log 2>&1 || exit $?
echo "=== k3prof done" >&2
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc "$c" --output-format csv -d "gpurun_out/k3pmc_$c" -o run \
    -- python bench.py --steps 2 --warmup 1 "${args[@]}" > "gpurun_out/k3pmc_$c.log" 2>&1 || exit $?
  echo "=== $c done" >&2
done
