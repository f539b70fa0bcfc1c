#!/bin/bash
# Round 4: the string pass with its five type counts packed in one word (cur) against the
# previous build (gpurun_ab/lib_prevstr.so): string-pass tests, the kernel alone (plan stream,
# DQ_PLAN_SIDE=0) under rocprofv3, then C5 alternated.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_profiles.py \
  tests/test_gpu_heap_tail.py tests/test_gpu_profiles_c5.py > gpurun_out/r04_strab_tests.log 2>&1
st=$?; tail -2 gpurun_out/r04_strab_tests.log; [ $st = 0 ] || exit $st
for v in cur prevstr; do
  lib=""; [ $v = prevstr ] && lib=gpurun_ab/lib_prevstr.so
  DQ_PLAN_SIDE=0 DEEQU_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_strab_prof_$v -o run \
    --output-format csv -- python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r04_strab_prof_$v.log 2>&1 || exit $?
  python - $v <<'PY'
import csv, sys
for r in csv.DictReader(open("gpurun_out/r04_strab_prof_%s/run_kernel_stats.csv" % sys.argv[1])):
    if "string_pass" in r["Name"]:
        print(sys.argv[1], r["Name"][:40], r["Calls"], "%.1f us avg, %.1f min" % (float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
done
for r in 1 2; do
  for v in prevstr cur; do
    lib=""; [ $v = prevstr ] && lib=gpurun_ab/lib_prevstr.so
    DEEQU_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r04_strab_$v.log 2>&1 || exit $?
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_strab_$v.log)"
  done
done
find gpurun_out -name "*kernel_trace.csv" -delete
