#!/bin/bash
# Same-box A/B/n of library builds (tools/build_variant.sh): the bench alternated over VARIANTS
# for ROUNDS rounds; prints ms_per_step and the headline kernel time of each run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-A B}; do
    DEEQU_AMD_LIB=$PWD/gpurun_ab/lib_$v.so timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/abn_${v}_$i.log 2>&1 || { echo "FAIL $v $i"; tail -3 gpurun_out/abn_${v}_$i.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/abn_${v}_$i.log').read().strip().split('\n')[-1]);print('$v',$i,round(d['ms_per_step'],3),round(d.get('roofline',{}).get('kernel_ms',0),3), d.get('scan_without_hll',{}).get('kernel_ms'))"
  done
done
