#!/bin/bash
# One gpurun session: partition/freq parity on the candidate builds, then a same-box C4 A/B.
mkdir -p gpurun_out
for L in f1; do
timeout -k 10 300 env DEEQU_AMD_LIB=gpurun_ab/lib_$L.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py > gpurun_out/pt_$L.log 2>&1 || { tail -5 gpurun_out/pt_$L.log; exit 1; }
tail -1 gpurun_out/pt_$L.log
done
WL=c4 STEPS=5 LIBS="f0 f1 f0 f1 f0 f1 f0 f1" bash tools/wlab.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu_final.log 2>&1 || { tail -5 gpurun_out/r02_pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/r02_pytest_gpu_final.log
