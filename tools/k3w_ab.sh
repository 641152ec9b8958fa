#!/bin/bash
# (round 6: no measurable change, not kept; the knob TCBEE_K3_WIDE_FRAMES is not in the tree)
# k_count's 16 records per lane from 16384 frames on (ab/ab_wt_new, the product) vs from
# 16M (ab/ab_wt_w16m: tools/lib_ab.sh build wt:w16m with
# HIPEXTRA=-DTCBEE_K3_WIDE_FRAMES=16777216): config 2 per step (tools/c2_ab.sh), and a
# 4M-frame IMIX batch (tools/k1_sweep.py) where the two differ too.
set -u
NAMES="wt_w16m wt_new" PAIRS=4 timeout -k 10 400 bash tools/c2_ab.sh || exit 1
NAMES="wt_w16m" PAIRS=2 timeout -k 10 400 bash tools/ab_multi.sh --workloads imix10k --frames 4000000 --cap-mult 1.04 || exit 1
