#!/bin/bash
# Round-end measurement, part B: HBM traffic (FETCH_SIZE / WRITE_SIZE, one pass each) of C2, C4,
# C5 and C3, stamped with the kernel-source digest the bench lines check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03f}
WL=c2 KERNEL='dq_scan' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c5 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
WL=c3 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
find gpurun_out -path "*pmct_*" -name "*counter_collection.csv" -delete
echo "PART B DONE"
