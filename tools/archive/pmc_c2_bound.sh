#!/bin/bash
# C2 bound evidence for DESIGN §5: instruction-class and stall counters of the fused scan kernels
# (one rocprofv3 --pmc pass per group), plus the per-instruction issue costs of the card
# (tools/ubench/valu_rates.hip).  Any failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
WL=c2 KERNEL=dq_scan_fast_kernel TAG=${TAG}_c2bound \
  PASSES="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_CVT,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" \
  BENCH_ARGS="--e2e-batch-rows 0" bash tools/pmc_kernel.sh || exit $?
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/ubench/valu_rates.hip -o /tmp/valu_rates && \
  timeout -k 10 120 /tmp/valu_rates > gpurun_out/valu_rates_${TAG}.txt 2>&1; tail -40 gpurun_out/valu_rates_${TAG}.txt
