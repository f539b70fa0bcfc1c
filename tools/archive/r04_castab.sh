#!/bin/bash
# Round 4: cast kernel with the next step's offsets prefetched (default) against without
# (gpurun_ab/lib_nopipe.so): cast tests, then C5 alternated, then per-kernel stats of each.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_profiles.py \
  tests/test_gpu_heap_tail.py tests/test_gpu_profiles_c5.py > gpurun_out/r04_castab_tests.log 2>&1
st=$?; tail -2 gpurun_out/r04_castab_tests.log; [ $st = 0 ] || exit $st
for r in 1 2; do
  for v in cur nopipe; do
    lib=""; [ $v = nopipe ] && lib=gpurun_ab/lib_nopipe.so
    DEEQU_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r04_castab_$v.log 2>&1 || exit $?
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_castab_$v.log)"
  done
done
for v in cur nopipe; do
  lib=""; [ $v = nopipe ] && lib=gpurun_ab/lib_nopipe.so
  DEEQU_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_castab_prof_$v -o run \
    --output-format csv -- python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r04_castab_prof_$v.log 2>&1 || exit $?
  python - $v <<'PY'
import csv, sys
for r in csv.DictReader(open("gpurun_out/r04_castab_prof_%s/run_kernel_stats.csv" % sys.argv[1])):
    if "cast_utf8" in r["Name"] or "string_pass" in r["Name"] or "small_kernel" in r["Name"]:
        print(sys.argv[1], r["Name"][:40], r["Calls"], "%.1f us avg, %.1f min" % (float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
done
find gpurun_out -name "*kernel_trace.csv" -delete
