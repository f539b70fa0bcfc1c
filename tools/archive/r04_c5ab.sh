#!/bin/bash
# Round 4: the profiler's GPU tests on the working tree, then C5 with the fused string pass on the
# plan's side stream (default) against the plan's own stream (DQ_PLAN_SIDE=0), alternated.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_profiles_c5.py \
    tests/test_gpu_profiles.py tests/test_gpu_heap_tail.py tests/test_gpu_parity_r2.py > gpurun_out/r04_c5ab_tests.log 2>&1
  st=$?; tail -2 gpurun_out/r04_c5ab_tests.log; [ $st = 0 ] || exit $st
fi
for r in 1 2; do
  for side in 1 0; do
    DQ_PLAN_SIDE=$side timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r04_c5ab_$side.log 2>&1 || exit $?
    echo "side=$side $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_c5ab_$side.log)"
  done
done
for side in 1 0; do
  DQ_PLAN_SIDE=$side timeout -k 10 200 python -u bench.py --workload c1 --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/r04_c1ab_$side.log 2>&1 || exit $?
  echo "c1 side=$side $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_c1ab_$side.log)"
done
if [ "${SPANS:-1}" = 1 ]; then
  SPANS=1 timeout -k 10 300 python -u tools/prof_host.py c5 > gpurun_out/r04_spans_c5b.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r04_spans_c5b.txt | tail -20
fi
if [ "${C4TRACE:-1}" = 1 ]; then  # C4 kernel timeline: where the step's non-kernel time goes
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04_c4trace -o run --output-format csv \
    -- python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04_c4trace.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_c4trace.log
fi
