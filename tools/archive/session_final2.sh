#!/bin/bash
# After the last kernel change: frequency tests, C4 bench + kernel trace, then PMC traffic.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_freq_partition.py \
  tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py tests/test_gpu_configs.py tests/test_gpu_table_hash.py \
  tests/test_gpu_distributed.py tests/test_gpu_sharded.py > gpurun_out/f2_tests.log 2>&1
st=$?; tail -2 gpurun_out/f2_tests.log; [ $st -eq 0 ] || exit $st
TAG=r03h WL="c4" bash tools/gpu_workloads.sh | tail -3 || exit 1
TAG=r03h bash tools/final_b.sh
