#!/bin/bash
# Round-6 GPU sessions.  PART=tests: a subset of the GPU tests (TESTS) in one pytest process;
# PART=ab: same-box A/B of environment knobs (tools/r05_envab.sh; VARIANTS / WL / STEPS);
# PART=c2pmc: the C2 scan kernels' issue / wait counters (one rocprofv3 --pmc pass per group).
# PART=bench: bench lines (BENCH_SET="name:--workload,c4,..."), one process each.
# Parts run in the order given (PARTS="tests ab"); any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06}
for P in ${PARTS:-tests}; do
  case $P in
    tests)
      timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 600 --timeout-method thread \
        > gpurun_out/${TAG}_tests.log 2>&1
      st=$?
      grep -E "passed|failed|error" gpurun_out/${TAG}_tests.log | tail -5
      [ $st -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit $st; } ;;
    ab)
      bash tools/r05_envab.sh || exit $? ;;
    ab2)  # a second A/B set: WL2 / VARIANTS2 / STEPS2
      WL=$WL2 VARIANTS=$VARIANTS2 STEPS=${STEPS2:-3} BENCH_ARGS=${BENCH_ARGS2:-${BENCH_ARGS:-}} bash tools/r05_envab.sh || exit $? ;;
    prof)  # kernel trace + stats of one bench command (PROF_ARGS, "," for spaces), PROF_ENV "A=1,B=2"
      env $(echo "${PROF_ENV:-}" | tr ',' ' ') timeout -k 10 ${PLIMIT:-400} rocprofv3 --kernel-trace --stats \
        -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 -u bench.py $(echo "$PROF_ARGS" | tr ',' ' ') \
        > gpurun_out/${TAG}_prof.log 2>&1
      st=$?
      tail -c 1200 gpurun_out/${TAG}_prof.log
      f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
      [ -n "$f" ] && cp "$f" gpurun_out/${TAG}_kernel_stats.csv && cut -d, -f1-8 gpurun_out/${TAG}_kernel_stats.csv | head -16
      find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
      [ $st -ne 0 ] && { echo "STOP prof (exit $st)"; exit $st; } ;;
    bench)  # one bench line per BENCH_SET entry ("name:args with , for spaces")
      for b in ${BENCH_SET:-c2:}; do
        name=${b%%:*}; a=$(echo "${b#*:}" | tr ',' ' ')
        timeout -k 10 ${BLIMIT:-400} python -u bench.py $a > gpurun_out/${TAG}_bench_$name.log 2>&1
        st=$?
        tail -c 1500 gpurun_out/${TAG}_bench_$name.log
        [ $st -ne 0 ] && { echo "STOP bench $name (exit $st)"; exit $st; }
      done ;;
    c2pmc)
      WL=c2 KERNEL=dq_scan_fast_kernel TAG=$TAG TL=240 \
        PASSES="SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU2,GRBM_GUI_ACTIVE;SQ_THREAD_CYCLES_VALU,SQ_BUSY_CU_CYCLES,SQ_ACTIVE_INST_LDS,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_ACTIVE_INST_SCA,SQ_WAVES,SQ_INSTS_VMEM_RD,GRBM_GUI_ACTIVE" \
        bash tools/pmc_kernel.sh || exit $? ;;
  esac
done
echo "SESSION DONE"
