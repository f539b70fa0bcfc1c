#!/bin/bash
# A/B: the same bench with two builds of the library, alternated, in one box session.
# Baseline build (untracked; .so files travel with gpurun):
#   git archive <rev> deequ_amd/csrc include | tar -x -C /tmp/old && make -C /tmp/old/deequ_amd/csrc
#   mkdir -p gpurun_ab && cp /tmp/old/deequ_amd/libdeequ_amd.so gpurun_ab/lib_old.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export DEEQU_AMD_LIB=$PWD/gpurun_ab/lib_old.so; else unset DEEQU_AMD_LIB; fi
    timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/ab_${v}_$i.log 2>&1 || { echo "FAIL $v $i"; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab_${v}_$i.log').read().strip().split('\n')[-1]);print('$v',$i,d['ms_per_step'],d.get('roofline',{}).get('kernel_ms'))"
  done
done
