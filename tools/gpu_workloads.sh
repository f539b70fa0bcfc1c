#!/bin/bash
# Secondary workloads (C3 HLL, C4 group-by): bench line + rocprofv3 kernel stats for each.
# Every GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
WL=${WL:-c3 c4}
for W in $WL; do
  timeout -k 10 400 python -u bench.py --workload $W --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} \
    > "$OUT/bench_${W}_$TAG.log" 2>&1
  st=$?; tail -2 "$OUT/bench_${W}_$TAG.log"
  if [ $st -ne 0 ]; then echo "STOP after bench $W (exit $st)"; exit $st; fi
  if [ "${PROF:-1}" = 1 ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${W}_$TAG" -o run --output-format csv \
      -- python -u bench.py --workload $W --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$OUT/prof_${W}_$TAG.log" 2>&1
    st=$?
    if [ $st -ne 0 ]; then echo "STOP after prof $W (exit $st)"; tail -5 "$OUT/prof_${W}_$TAG.log"; exit $st; fi
    f=$(find "$OUT/prof_${W}_$TAG" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/kernel_stats_${W}_$TAG.csv"
    cut -c1-160 "$OUT/kernel_stats_${W}_$TAG.csv" | head -8
  fi
done
echo "ALL DONE"
