#!/bin/bash
# Round-5 GPU session: a chosen subset of the GPU tests (TESTS), one pytest process, its own time
# limit; the log lands in gpurun_out/r05_tests_$TAG.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-a}
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/r05_tests_$TAG.log 2>&1
st=$?
grep -E "^\[|passed|failed|error" gpurun_out/r05_tests_$TAG.log | tail -20
exit $st
