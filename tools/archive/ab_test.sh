#!/bin/bash
# One pytest selection against several library builds (gpurun_ab/lib_<name>.so), same box.
# Usage: LIBS="base new" SEL="tests/x.py::t" bash tools/ab_test.sh
set -u
mkdir -p gpurun_out
for lib in $LIBS; do
  DEEQU_AMD_LIB=gpurun_ab/lib_$lib.so timeout -k 10 ${TL:-300} python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread $SEL > gpurun_out/abt_$lib.log 2>&1
  st=$?
  echo "$lib: exit $st: $(tail -1 gpurun_out/abt_$lib.log)"
  if [ $st -ge 124 ]; then exit $st; fi
done
