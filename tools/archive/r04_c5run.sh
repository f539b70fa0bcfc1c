set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_freq_small.py tests/test_gpu_heap_tail.py tests/test_gpu_profiles_c5.py tests/test_gpu_profiles.py > gpurun_out/r04_c5tests.log 2>&1
st=$?; tail -2 gpurun_out/r04_c5tests.log; grep -E "^FAILED" gpurun_out/r04_c5tests.log | head -5; [ $st -lt 124 ] || exit $st
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_c5prof2 -o run --output-format csv -- python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04_c5prof2.log 2>&1
st=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04_c5prof2.log; exit $st
