#!/bin/bash
set -u
LIBS="g0 h1 h2 g0 h1 h2" WL=c4 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|stage_part|STOP|FAILED"
for v in h1; do
  DEEQU_AMD_LIB=gpurun_ab/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_freq_partition.py "tests/test_gpu_configs.py::test_c4_scale_partition_group_by" > gpurun_out/ab5_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/ab5_$v.log)"
done
