#!/bin/bash
# Round-6 measurement in GPU sessions (on the committed build): PART=a -> smoke + the whole GPU
# suite + the default bench + its kernel trace (tools/gpu_check.sh); PART=b -> every secondary
# workload and C4 key shape, a bench line and a kernel-stats profile each; PART=c -> the HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE, one per pass) of C2, C4 (digits, alnum, uuid), C5 and
# C3, stamped with the kernel-source digest.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r06}
case "${PART:-a}" in
  a) TAG=$TAG bash tools/gpu_check.sh || exit $? ;;
  b)
    for v in ${SET:-c1: c3: c4: c4_alnum:--c4-keys,alnum c4_uuid:--c4-keys,uuid c4_pair:--c4-keys,pair c4_pair64:--c4-keys,pair64 c5:}; do
      name=${v%%:*}; args=$(echo "${v#*:}" | tr ',' ' '); W=${name%%_*}
      timeout -k 10 400 python -u bench.py --workload $W --steps ${STEPS:-5} --warmup 2 $args \
        > "$OUT/bench_${name}_$TAG.log" 2>&1
      st=$?; tail -c 600 "$OUT/bench_${name}_$TAG.log"; echo
      if [ $st -ne 0 ]; then echo "STOP after bench $name (exit $st)"; exit $st; fi
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${name}_$TAG" -o run --output-format csv \
        -- python3 -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline $args > "$OUT/prof_${name}_$TAG.log" 2>&1
      st=$?
      if [ $st -ne 0 ]; then echo "STOP after prof $name (exit $st)"; tail -5 "$OUT/prof_${name}_$TAG.log"; exit $st; fi
      f=$(find "$OUT/prof_${name}_$TAG" -name "*kernel_stats.csv" | head -1)
      cp "$f" "$OUT/kernel_stats_${name}_$TAG.csv"
      find "$OUT/prof_${name}_$TAG" -name "*kernel_trace.csv" -delete
    done ;;
  c)
    WL=c2 KERNEL='dq_scan' STEPS=1 TAG=${TAG} bash tools/pmc_traffic.sh || exit $?
    WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=${TAG} bash tools/pmc_traffic.sh || exit $?
    WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=${TAG}_alnum BENCH_ARGS="--c4-keys alnum" bash tools/pmc_traffic.sh || exit $?
    WL=c4 KERNEL='dq::dq_freq' STEPS=1 TAG=${TAG}_uuid BENCH_ARGS="--c4-keys uuid" bash tools/pmc_traffic.sh || exit $?
    WL=c5 KERNEL='dq::' STEPS=1 TAG=${TAG} bash tools/pmc_traffic.sh || exit $?
    WL=c3 KERNEL='dq::' STEPS=1 TAG=${TAG} bash tools/pmc_traffic.sh || exit $?
    find "$OUT" -path "*pmct_*" -name "*counter_collection.csv" -delete ;;
esac
find "$OUT" -name "*kernel_trace.csv" -delete
echo "PART ${PART:-a} DONE"
