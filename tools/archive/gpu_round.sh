#!/bin/bash
# Round measurement in one GPU session: smoke, GPU tests, the default bench + its rocprofv3 kernel
# trace, every secondary workload (+ the C3 string variant) with its kernel trace, then the PMC
# passes (FETCH/WRITE traffic, VALU/clock) of the headline scan.  Each step has its own time
# limit; any failure ends the script.  Large raw profiler output is pruned at the end so the
# merged gpurun_out/ stays small.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
TAG=$TAG bash tools/gpu_check.sh || exit $?
TAG=$TAG WL="c1 c3 c4 c5" bash tools/gpu_workloads.sh || exit $?
TAG=${TAG}u WL=c3 BENCH_ARGS="--c3-type utf8" bash tools/gpu_workloads.sh || exit $?
TAG=$TAG bash tools/pmc_round.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -path "*pmck_*" -name "*counter_collection.csv" -delete
echo "ROUND DONE"
