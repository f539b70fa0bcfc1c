#!/bin/bash
# Round 4: frequency GPU tests on the working tree's library, then per-kernel C4 A/B of the
# gpurun_ab/ builds in LIBS, then the stage phase timing (lib_sprof, -DDQ_STAGE_PROF).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest --maxfail=5 -v -s --timeout 200 --timeout-method thread ${TESTFILES:-tests/test_gpu_freq_import.py tests/test_gpu_freq_small.py \
    tests/test_gpu_table_hash.py tests/test_gpu_freq_partition.py tests/test_gpu_frequencies.py tests/test_gpu_freq_paths.py \
    tests/test_gpu_profiles_c5.py tests/test_gpu_profiles.py tests/test_gpu_distributed.py tests/test_gpu_sharded.py \
    tests/test_gpu_configs.py} > gpurun_out/r04_tests.log 2>&1
  st=$?; tail -3 gpurun_out/r04_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04_tests.log | head -5
  [ $st -lt 124 ] || exit $st   # test failures: still time the kernels; a fault / abort / time limit: stop
fi
LIBS="${LIBS:-base n1}" WL=${WL:-c4} bash tools/kprof_ab.sh 2>&1 | tee gpurun_out/r04_kprof.txt | grep -E "ms_per_step|part_kernel|agg_packed|stage_part|insert|STOP|FAILED" || exit 1
for sp in ${SPROF:-sprof}; do
  [ -f gpurun_ab/lib_$sp.so ] || continue
  DEEQU_AMD_LIB=gpurun_ab/lib_$sp.so timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 \
    --no-cpu-baseline > gpurun_out/r04_$sp.log 2>&1
  st=$?; echo "$sp:"; grep stage_prof gpurun_out/r04_$sp.log | tail -2; [ $st -eq 0 ] || exit $st
done
if [ -f gpurun_ab/lib_sdiag.so ] && [ "${SDIAG:-0}" = 1 ]; then
  DEEQU_AMD_LIB=gpurun_ab/lib_sdiag.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-side-passes \
    --no-cpu-baseline > gpurun_out/r04_sdiag.log 2>&1
  st=$?; echo "sdiag:"; grep scan_diag gpurun_out/r04_sdiag.log | sort | uniq -c | head -8; exit $st
fi
