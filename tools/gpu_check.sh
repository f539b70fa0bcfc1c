#!/bin/bash
# One GPU session: smoke -> GPU tests -> short bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; anything but success / ordinary test failures
# (pytest exit 1) ends the script so nothing else touches a possibly faulted GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
STEPS=${STEPS:-smoke,tests,bench,prof}

ok_or_stop() {  # $1 = exit status, $2 = step name, $3 = allowed non-zero (optional)
  local st=$1
  if [ "$st" -ne 0 ] && [ "$st" -ne "${3:-0}" ]; then
    echo "STOP after $2 (exit $st)"; exit "$st"
  fi
}

if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  st=$?; tail -3 "$OUT/smoke_$TAG.log"; ok_or_stop $st smoke
fi
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  st=$?; tail -15 "$OUT/pytest_gpu_$TAG.log"; ok_or_stop $st tests 1
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python -u bench.py --steps ${BENCH_STEPS:-10} --warmup 3 ${BENCH_ARGS:-} \
    > "$OUT/bench_$TAG.log" 2>&1
  st=$?; tail -3 "$OUT/bench_$TAG.log"; ok_or_stop $st bench
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv \
    -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side-passes > "$OUT/prof_$TAG.log" 2>&1
  st=$?; tail -3 "$OUT/prof_$TAG.log"; ok_or_stop $st prof
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$TAG.csv" \; 2>/dev/null
  head -20 "$OUT/kernel_stats_$TAG.csv" 2>/dev/null
fi
echo "ALL DONE"
