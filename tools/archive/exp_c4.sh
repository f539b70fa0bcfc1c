#!/bin/bash
# C4 iteration: frequency tests, then the C4 bench and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-exp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py tests/test_gpu_distributed.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/c4_tests_$TAG.log 2>&1
st=$?; tail -1 gpurun_out/c4_tests_$TAG.log; [ $st -eq 0 ] || exit $st
TAG=$TAG WL=c4 bash tools/gpu_workloads.sh || exit $?
find gpurun_out -name "*kernel_trace.csv" -delete
