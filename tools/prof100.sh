#!/bin/bash
# kernel-trace profile of one 100M-frame config-3 sweep (flows on)
rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof100 -o run -- python tools/k1_sweep.py --fpl 2 --workloads imix10k --rounds 1 --iters 5 --flows-only "$@"
