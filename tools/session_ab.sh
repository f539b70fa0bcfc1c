mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_scan.py tests/test_gpu_c1.py tests/test_gpu_parity.py > gpurun_out/pt_nt.log 2>&1 || { tail -5 gpurun_out/pt_nt.log; exit 1; }
tail -1 gpurun_out/pt_nt.log
for W in c1 c2; do timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ntb_$W.log 2>&1 || exit 1; echo "$W $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ntb_$W.log)"; done
for L in pb4 pb8; do timeout -k 10 200 env DEEQU_AMD_LIB=gpurun_ab/lib_$L.so python -u -m pytest -x -q --timeout 90 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py > gpurun_out/pt_$L.log 2>&1 || { tail -5 gpurun_out/pt_$L.log; exit 1; }; tail -1 gpurun_out/pt_$L.log; done
WL=c4 LIBS="base pb4 pb8 base pb4 pb8" bash tools/wlab.sh
