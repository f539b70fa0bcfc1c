#!/bin/bash
# Round-5 measurement in GPU sessions (on the committed build): PART=a -> smoke + the whole GPU
# suite + the default bench + its kernel trace; PART=b -> every secondary workload with its
# kernel trace; PART=c -> the HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one per pass) of C2,
# C4, C5 and C3 stamped with the kernel-source digest.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05}
case "${PART:-a}" in
  a) TAG=$TAG bash tools/gpu_check.sh || exit $? ;;
  b) TAG=$TAG WL="${WL:-c1 c3 c4 c5}" bash tools/gpu_workloads.sh || exit $? ;;
  c)
    WL=c2 KERNEL='dq_scan' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
    WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
    WL=c5 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
    WL=c3 KERNEL='dq::' STEPS=1 TAG=$TAG bash tools/pmc_traffic.sh || exit $?
    find gpurun_out -path "*pmct_*" -name "*counter_collection.csv" -delete ;;
  d)  # the key-hash exchange's receiver at C4 scale: 8 parts of an 8e7-row table imported
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_import_$TAG -o run --output-format csv \
      -- python -u -m pytest -v -s --timeout 300 --timeout-method thread \
      "tests/test_gpu_freq_import.py::test_c4_scale_partition_import" > gpurun_out/prof_import_$TAG.log 2>&1 || exit $?
    grep -E "c4 import|passed|failed" gpurun_out/prof_import_$TAG.log ;;
esac
find gpurun_out -name "*kernel_trace.csv" -delete
echo "PART ${PART:-a} DONE"
