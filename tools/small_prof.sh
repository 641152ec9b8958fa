#!/bin/bash
rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/smallprof -o run -- python tools/k1_sweep.py --frames 1000000 --fpl 2 --workloads 64B1 --rounds 1 --iters 20
