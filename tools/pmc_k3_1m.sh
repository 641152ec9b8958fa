#!/bin/bash
# K3 mode 1 (k_count_chunk2 + k_count_bucket): what bounds it. LEG=1M (default): the
# whole 1M-flow trace (--config4 --shard contig: 125M IMIX frames); LEG=share: one
# GPU's flow-hash share at N=8 (--config4 --virtual-world 8); outputs
# gpurun_out/k3pmc_<LEG>_<pass>. Separate
# --pmc passes (at most 8 SQ_ / 4 TCC_ counters each), each its own short run
# under a hard limit (MI355X_MICROARCH.md: counters in their own runs).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
case ${LEG:-1M} in
  share) legargs=(--config4 --virtual-world 8) ;;
  c3) legargs=() ;;  # config 3 (K3 mode 0; K1 counters in the same passes)
  *) legargs=(--config4 --shard contig) ;;
esac
args=(--steps 2 --warmup 1 --no-cpu --no-extra --sample-check "${legargs[@]}")
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/${name/k3pmc_/k3pmc_${LEG:-1M}_}" -o run \
    -- python bench.py "${args[@]}" > "gpurun_out/${name/k3pmc_/k3pmc_${LEG:-1M}_}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
pass k3pmc_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS
pass k3pmc_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES \
  TCC_HIT_sum TCC_MISS_sum
pass k3pmc_fetch FETCH_SIZE
pass k3pmc_write WRITE_SIZE
