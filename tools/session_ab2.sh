#!/bin/bash
# GPU session: lane-queue aggregation variant -- parity on the partition tests, then per-kernel A/B.
set -u
mkdir -p gpurun_out
DEEQU_AMD_LIB=gpurun_ab/lib_q1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py tests/test_gpu_configs.py > gpurun_out/pt_q1.log 2>&1 || { tail -30 gpurun_out/pt_q1.log; exit 1; }
tail -1 gpurun_out/pt_q1.log
LIBS="q0 q1 q0 q1" bash tools/kprof_ab.sh
