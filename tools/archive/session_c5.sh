#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_profiles.py \
  tests/test_gpu_profiles_c5.py tests/test_gpu_sharded.py > gpurun_out/c5_tests.log 2>&1
st=$?; tail -2 gpurun_out/c5_tests.log; [ $st -eq 0 ] || exit $st
for mode in 1 0 1 0; do
  DEEQU_AMD_PROFILE_SERIAL=$mode timeout -k 10 300 python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/c5_serial$mode.log 2>&1 || exit $?
  echo "serial=$mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_serial$mode.log)"
done
