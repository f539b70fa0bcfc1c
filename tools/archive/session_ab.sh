#!/bin/bash
# One gpurun session: frequency-path parity on the in-tree build, then the C2 A/B (tools/c2ab.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py tests/test_gpu_configs.py tests/test_gpu_distributed.py > gpurun_out/pt_split.log 2>&1 || { tail -30 gpurun_out/pt_split.log; exit 1; }
tail -1 gpurun_out/pt_split.log
bash tools/c2ab.sh
