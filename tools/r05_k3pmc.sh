#!/bin/bash
# Round 5: K3 mode-1 PMC (tools/pmc_k3_1m.sh) on the N=8 share and the whole 1M-flow trace
set -u
K3ARGS="--config4 --virtual-world 8" bash tools/pmc_k3_1m.sh || exit $?
for p in sq lds fetch write; do rm -rf gpurun_out/k3pmc_share_$p; mv gpurun_out/k3pmc_$p gpurun_out/k3pmc_share_$p; done
K3ARGS="--config4 --shard contig" bash tools/pmc_k3_1m.sh || exit $?
