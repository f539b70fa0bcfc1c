#!/bin/bash
# One GPU session: the whole suite on the in-tree build, VALU issue/latency microbenchmark, the C2
# A/B, the aggregation lane-queue A/B.
set -u
mkdir -p gpurun_out
tools/gpu_final.sh r03c || exit 1
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/ubench/valu_rates.hip -o /tmp/valu_rates && \
  timeout -k 10 120 /tmp/valu_rates > gpurun_out/valu_rates_r03.txt 2>&1 || exit 1
LIBS="c0 c1 c4 c5 c0 c1 c4" bash tools/c2ab.sh || exit 1
bash tools/session_ab2.sh
