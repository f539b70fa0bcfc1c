#!/bin/bash
# Same-box A/B of C4 variants: library builds in gpurun_ab/ x table load factors.
mkdir -p gpurun_out
for lib in ${LIBS:-def}; do
  for load in ${LOADS:-0.92 0.46}; do
    DEEQU_AMD_LIB=gpurun_ab/lib_$lib.so DQ_FREQ_PART_LOAD=$load timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/c4ab_${lib}_$load.log 2>&1 || exit $?
    echo "$lib $load $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4ab_${lib}_$load.log)"
  done
done
