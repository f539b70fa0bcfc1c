#!/bin/bash
# Round 4, the verdict's measurement items on one GPU box: bench.py's 2-rank gloo path for c1-c5,
# C4 at 1e9 rows against torch.unique, C3's whole 1e9 x 64 job (8 batches, full_job), C4 with
# non-digit keys, and C5 with per-kernel stats.  Logs under gpurun_out/r04_*.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, time limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/r04_$name.log 2>&1
  local st=$?
  echo "$name: exit $st"; grep -E '^\{|passed|failed|FAILED|Error' gpurun_out/r04_$name.log | cut -c1-400 | tail -4
  [ $st -lt 124 ] || exit $st
}
if [ "${RANKS:-1}" = 1 ]; then
  run ranks 700 python -u -m pytest -v -s --timeout 320 --timeout-method thread tests/test_gpu_bench_ranks.py
fi
if [ "${C4FULL:-1}" = 1 ]; then
  run c4full 400 python -u -m pytest -v -s --timeout 380 --timeout-method thread tests/test_gpu_c4_full.py
fi
if [ "${C3FULL:-1}" = 1 ]; then
  run c3full 400 python -u bench.py --workload c3 --c3-batches 8 --steps 2 --warmup 1 --no-cpu-baseline
fi
if [ "${C4ALNUM:-1}" = 1 ]; then
  run c4alnum 300 python -u bench.py --workload c4 --c4-keys alnum --steps 2 --warmup 1 --no-cpu-baseline
fi
if [ "${C5PROF:-1}" = 1 ]; then
  run c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_c5prof -o run --output-format csv \
    -- python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
fi
