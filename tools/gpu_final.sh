#!/bin/bash
# Round-end check of the committed default build: the whole GPU suite, then smoke.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu_final.log 2>&1 || { tail -5 gpurun_out/r02_pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/r02_pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke_final.log 2>&1 && tail -1 gpurun_out/r02_smoke_final.log
