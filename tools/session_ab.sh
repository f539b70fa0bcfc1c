#!/bin/bash
# One gpurun session: the whole GPU suite on the in-tree build, then a same-box C4 A/B.
set -u
mkdir -p gpurun_out
tools/gpu_final.sh ${TAG:-r03b} || exit 1
WL=c4 STEPS=5 LIBS="${LIBS:-a0 a1 a2 a3 a0 a1 a2 a3}" bash tools/wlab.sh
