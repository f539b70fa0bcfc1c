#!/bin/bash
# Round 5: per-kernel C4 timing of the gpurun_ab/ builds in LIBS (tools/kprof_ab.sh), the stage
# phase profile of lib_sprof, and the last step's kernel timeline of the first build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="${LIBS:-base}" WL=${WL:-c4} STEPS=${STEPS:-2} bash tools/kprof_ab.sh 2>&1 | tee gpurun_out/r05_kprof.txt | grep -E "ms_per_step|part_kernel|agg_packed|stage_part|STOP|FAILED" || exit 1
first=${LIBS%% *}
f=$(find gpurun_out/kprof_$first -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 tools/timeline.py "$f" "${MARK:-dq_freq_stage_part}" 5 > gpurun_out/r05_timeline_$first.txt 2>&1
tail -3 gpurun_out/r05_timeline_$first.txt
if [ -f gpurun_ab/lib_sprof.so ] && [ "${SPROF:-1}" = 1 ]; then
  DEEQU_AMD_LIB=gpurun_ab/lib_sprof.so timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 \
    --no-cpu-baseline > gpurun_out/r05_sprof.log 2>&1
  st=$?; grep stage_prof gpurun_out/r05_sprof.log | tail -2; [ $st -eq 0 ] || exit $st
fi
find gpurun_out -name "*kernel_trace.csv" -size +20M -delete
echo DONE
