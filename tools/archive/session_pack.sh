#!/bin/bash
# Packed digit-key records: the frequency tests, then C4 timing (HIP events + kernel stats).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_freq_partition.py \
  tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py "tests/test_gpu_configs.py::test_c4_scale_partition_group_by" \
  > gpurun_out/pk_tests.log 2>&1
st=$?; tail -4 gpurun_out/pk_tests.log; [ $st -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pk_tests.log | head -20; exit $st; }
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pk_c4.log 2>&1
st=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/pk_c4.log; [ $st -eq 0 ] || { tail -5 gpurun_out/pk_c4.log; exit $st; }
DQ_FREQ_PACK=0 timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pk_c4_raw.log 2>&1
st=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/pk_c4_raw.log; [ $st -eq 0 ] || exit $st
mkdir -p gpurun_ab && cp deequ_amd/libdeequ_amd.so gpurun_ab/lib_x0.so && LIBS=x0 WL=c4 bash tools/kprof_ab.sh 2>&1 | tail -8
