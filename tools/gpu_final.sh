#!/bin/bash
# Round-end check of the committed default build: the whole GPU suite, then smoke.
# Usage: tools/gpu_final.sh [tag]   (logs: gpurun_out/<tag>_pytest_gpu.log, <tag>_smoke.log)
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log
