#!/bin/bash
# Round-3 measurement in one GPU session (on the committed build): smoke + the whole GPU suite +
# the default bench + its kernel trace (tools/gpu_check.sh), every secondary workload with its
# kernel trace, then the HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one per pass) of C2, C4,
# C5 and C3 stamped with the kernel-source digest.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
TAG=$TAG bash tools/gpu_check.sh || exit $?
TAG=$TAG WL="c1 c3 c4 c5" bash tools/gpu_workloads.sh || exit $?
WL=c2 KERNEL='dq_scan' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c5 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c3 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -path "*pmct_*" -name "*counter_collection.csv" -delete
echo "ROUND DONE"
