#!/bin/bash
# Round-end measurement, part A: smoke + full GPU suite + default bench + kernel trace, then the
# secondary workloads (bench line + kernel trace each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03f}
TAG=$TAG bash tools/gpu_check.sh || exit $?
TAG=$TAG WL="c1 c3 c4 c5" bash tools/gpu_workloads.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
echo "PART A DONE"
