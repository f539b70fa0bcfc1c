#!/bin/bash
# Round PMC evidence (one rocprofv3 --pmc pass per counter group, never combined with tracing):
# HBM traffic per step of C2 / C3 / C4 / C5, LDS bank conflicts of the HLL register updates (C2
# fused scan, C3 string HLL), LDS + L2 atomics of the C4 group-by kernels.  Any failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
WL=c2 KERNEL='dq_scan' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c5 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c3 KERNEL='dq::' STEPS=1 TAG=$TAG BENCH_ARGS="--c3-rows 125000000" bash tools/pmc_traffic.sh || exit $?
WL=c2 KERNEL=dq_scan_fast_kernel TAG=$TAG \
  PASSES="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_LDS_ATOMIC_RETURN,SQ_LDS_ADDR_CONFLICT,GRBM_GUI_ACTIVE,SQ_WAVES" \
  bash tools/pmc_kernel.sh || exit $?
WL=c3 KERNEL=dq_hll_kernel TAG=${TAG}u BENCH_ARGS="--c3-type utf8 --c3-rows 125000000" \
  PASSES="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_LDS_ATOMIC_RETURN,SQ_LDS_ADDR_CONFLICT,GRBM_GUI_ACTIVE,SQ_WAVES" \
  bash tools/pmc_kernel.sh || exit $?
for K in dq_freq_stage_part_kernel dq_freq_part_kernel dq_freq_agg_region_kernel; do
  WL=c4 KERNEL=$K TAG=${TAG}_$K \
    PASSES="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_LDS_ATOMIC_RETURN,SQ_INSTS_LDS_ATOMIC,GRBM_GUI_ACTIVE,SQ_WAVES;TCC_ATOMIC_sum,TCC_EA0_ATOMIC_sum" \
    bash tools/pmc_kernel.sh || exit $?
done
find gpurun_out -path "*pmck_*" -name "*counter_collection.csv" -delete
find gpurun_out -path "*pmct_*" -name "*counter_collection.csv" -delete
echo "PMC DONE"
