#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel stats of one bench workload for each library build in
# gpurun_ab/ (LIBS), summarised per kernel (avg ms) into gpurun_out/kprof_<lib>.txt.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-x0}; do
  D=gpurun_out/kprof_$lib
  DEEQU_AMD_LIB=gpurun_ab/lib_$lib.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv \
    -- python -u bench.py --workload ${WL:-c4} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $D.log 2>&1
  st=$?
  if [ $st -ge 124 ]; then echo "STOP $lib: exit $st (fault / abort / time limit)"; tail -3 $D.log; exit $st; fi
  if [ $st -ne 0 ]; then echo "FAILED $lib (exit $st: an exception, timing still in the trace)"; grep -v "^[WE]2026" $D.log | tail -2; fi
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "dq::" in r["Name"]]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
out = ["%s %-45s calls %4s avg %8.3f ms min %8.3f" % (sys.argv[2], r["Name"].split("(")[0][-45:], r["Calls"],
       float(r["AverageNs"]) / 1e6, float(r["MinNs"]) / 1e6) for r in rows[:6]]
print("\n".join(out))
PY
  grep -o '"ms_per_step": [0-9.]*' $D.log
done
