#!/bin/bash
# Kernel trace of one bench workload (WL), last step summarised: per-kernel busy time, idle gaps
# (tools/timeline.py on the dispatches from the last MARK on).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
D=gpurun_out/trace_${WL:-c5}
timeout -k 10 300 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 -u bench.py --workload ${WL:-c5} \
  --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $D.log 2>&1 || { tail -3 $D.log; exit 1; }
f=$(find $D -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" "${MARK:-dq_scan_fast}" ${MIN_GAP:-20} > gpurun_out/timeline_${WL:-c5}.txt
tail -3 gpurun_out/timeline_${WL:-c5}.txt
gzip -f "$f"
