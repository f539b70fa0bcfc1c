#!/bin/bash
# C4 variants, then C5 insert-kernel layout A/B, then the frequency tests on the default build.
set -u
LIBS="x4 x5 y2 y3 y4 y5 y6 y7 y8 z1" WL=c4 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|part_kernel|agg_packed|stage_part|STOP|FAILED" || exit 1
LIBS="x4 x5" WL=c5 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|insert|STOP|FAILED" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_freq_paths.py \
  tests/test_gpu_frequencies.py tests/test_gpu_profiles_c5.py tests/test_gpu_table_hash.py > gpurun_out/ab2_tests.log 2>&1
st=$?; tail -2 gpurun_out/ab2_tests.log; exit $st
