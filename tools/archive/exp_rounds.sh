#!/bin/bash
# Scan-grid sweep: the C2 bench at several DQ_SCAN_ROUNDS (whole rounds of resident workgroups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in ${ROUNDS:-1 2 3 4}; do
  DQ_SCAN_ROUNDS=$R timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/exp_rounds_$R.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/exp_rounds_$R.log') if l.startswith('{')][-1]);print('R=$R', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
