#!/bin/bash
set -u
mkdir -p gpurun_out
LIBS="c0 c6 c0 c6 c0 c6" bash tools/c2ab.sh || exit 1
TAG=r03 bash tools/pmc_c2_bound.sh
