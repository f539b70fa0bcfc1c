#!/bin/bash
set -u
LIBS="w0 w1 w2 w3" WL=c4 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|part_kernel|agg_packed|stage_part|STOP|FAILED" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_freq_partition.py \
  tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py "tests/test_gpu_configs.py::test_c4_scale_partition_group_by" \
  tests/test_gpu_table_hash.py > gpurun_out/ab3_tests.log 2>&1
st=$?; tail -2 gpurun_out/ab3_tests.log; exit $st
