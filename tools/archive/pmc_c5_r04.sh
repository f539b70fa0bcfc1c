set -u
for K in dq_freq_small_kernel dq_string_pass_kernel; do
  WL=c5 KERNEL=$K TAG=r04_$K TL=240 PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_IFETCH" bash tools/pmc_kernel.sh || exit $?
done
find gpurun_out -path "*pmck_*" -name "*counter_collection.csv" -delete
