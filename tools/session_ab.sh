set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_freq_partition.py tests/test_gpu_freq_paths.py tests/test_gpu_frequencies.py tests/test_gpu_configs.py > gpurun_out/pt_h1.log 2>&1 || { tail -20 gpurun_out/pt_h1.log; exit 1; }
tail -1 gpurun_out/pt_h1.log
WL=c4 STEPS=5 LIBS="h0 h1 h0 h1 h0 h1" bash tools/wlab.sh
