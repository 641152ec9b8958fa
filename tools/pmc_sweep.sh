#!/bin/bash
# HBM traffic of K1 on the 100M config-3 sweep (flows on): separate FETCH/WRITE passes
set -e
rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcs_fetch -o run -- python tools/k1_sweep.py --fpl 2 --workloads imix10k --rounds 1 --iters 2 --flows-only
rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcs_write -o run -- python tools/k1_sweep.py --fpl 2 --workloads imix10k --rounds 1 --iters 2 --flows-only
