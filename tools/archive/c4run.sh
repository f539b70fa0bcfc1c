mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 90 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py tests/test_gpu_profiles_c5.py > gpurun_out/pt_part.log 2>&1
st=$?; tail -5 gpurun_out/pt_part.log; [ $st -eq 0 ] || exit $st
DQ_FREQ_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/c4_part.log 2>&1
st=$?; tail -3 gpurun_out/c4_part.log; [ $st -eq 0 ] || exit $st
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4p -o run --output-format csv -- python -u bench.py --workload c4 --steps 2 --warmup 1 > gpurun_out/prof_c4p.log 2>&1
echo prof $?
