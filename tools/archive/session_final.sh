#!/bin/bash
# Cast change check (profiler tests + C5 kernel stats), then the PMC traffic passes (part B).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_profiles.py \
  tests/test_gpu_profiles_c5.py tests/test_gpu_parity_r2.py > gpurun_out/fin_tests.log 2>&1
st=$?; tail -2 gpurun_out/fin_tests.log; [ $st -eq 0 ] || exit $st
mkdir -p gpurun_ab && cp deequ_amd/libdeequ_amd.so gpurun_ab/lib_f0.so && LIBS=f0 WL=c5 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|cast|insert|string|STOP|FAILED"
bash tools/final_b.sh
