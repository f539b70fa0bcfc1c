#!/bin/bash
# Issue / wait breakdown of the three C4 partition-path kernels (one --pmc pass per kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for K in dq_freq_agg_region_kernel dq_freq_stage_part_kernel dq_freq_part_kernel; do
  WL=c4 KERNEL=$K TAG=stall_$K \
    PASSES="SQ_WAVE_CYCLES,SQ_WAIT_INST_LDS,SQ_WAIT_ANY,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_VMEM,SQ_INSTS_VALU,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE" \
    bash tools/pmc_kernel.sh || exit $?
done
find gpurun_out -path "*pmck_*" -name "*counter_collection.csv" -delete
