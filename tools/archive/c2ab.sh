set -u
mkdir -p gpurun_out
for lib in ${LIBS:-c0 c1 c2 c3 c4 c5 c0 c1 c4}; do
  DEEQU_AMD_LIB=gpurun_ab/lib_$lib.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-passes --e2e-batch-rows 0 > gpurun_out/c2ab_$lib.log 2>&1 || { echo "FAIL $lib $?"; tail -3 gpurun_out/c2ab_$lib.log; exit 1; }
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c2ab_$lib.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c2ab_$lib.log | head -1)"
done
