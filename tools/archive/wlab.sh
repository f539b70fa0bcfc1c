#!/bin/bash
# Same-box A/B of library builds in gpurun_ab/ on one bench workload (WL), alternated.
mkdir -p gpurun_out
for lib in ${LIBS:-new head}; do
  DEEQU_AMD_LIB=gpurun_ab/lib_$lib.so timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/wlab_${WL}_$lib.log 2>&1 || exit $?
  echo "$WL $lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wlab_${WL}_$lib.log)"
done
