#!/bin/bash
# C4 per-kernel A/B of library variants (gpurun_ab/lib_<x>.so), then the load-factor knob on x0.
set -u
LIBS="${LIBS:-x0 x1 x2 x3}" WL=c4 bash tools/kprof_ab.sh || exit $?
for load in; do
  DQ_FREQ_PART_LOAD=$load DEEQU_AMD_LIB=gpurun_ab/lib_x0.so timeout -k 10 200 python -u bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/c4_load_$load.log 2>&1 || exit $?
  echo "load $load: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_load_$load.log)"
done
