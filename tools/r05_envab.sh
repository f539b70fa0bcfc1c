#!/bin/bash
# Round 5: same-box A/B of environment knobs on one workload.  VARIANTS="name:ENV=V,ENV2=W name2:..."
# (":" alone = defaults).  Per variant: rocprofv3 kernel stats of bench.py (STEPS steps), the
# dq:: kernels' averages and the bench line's ms_per_step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; envs=${v#*:}
  D=gpurun_out/envab_$name
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv \
    -- python3 -u bench.py --workload ${WL:-c4} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $D.log 2>&1
  st=$?
  if [ $st -ge 124 ]; then echo "STOP $name: exit $st"; tail -3 $D.log; exit $st; fi
  [ $st -ne 0 ] && { echo "FAILED $name (exit $st)"; tail -3 $D.log; }
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$name" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "dq::" in r["Name"]]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print("%s %-48s calls %4s avg %8.3f ms min %8.3f" % (sys.argv[2], r["Name"].split("(")[0][-48:], r["Calls"],
          float(r["AverageNs"]) / 1e6, float(r["MinNs"]) / 1e6))
PY
  grep -o '"ms_per_step": [0-9.]*' $D.log
  find $D -name "*kernel_trace.csv" -delete
done
echo DONE
