set -u
cd "${GRAFT_REPO_ROOT}"
for v in old new; do
  if [ $v = old ]; then export DEEQU_AMD_LIB=$PWD/gpurun_ab/lib_old.so; else unset DEEQU_AMD_LIB; fi
  WL=c2 KERNEL=dq_scan_values_kernel TAG=ab$v PASSES="SQ_INSTS_VALU,SQ_INSTS_SALU,GRBM_GUI_ACTIVE,SQ_WAVES,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_INST_CYCLES_VMEM" bash tools/pmc_kernel.sh || exit 1
done
find gpurun_out -path "*pmck_*" -name "*counter_collection.csv" -delete
