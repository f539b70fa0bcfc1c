#!/bin/bash
# C4 group-by probe: growing row counts, sorted-bucket vs atomic path, each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for R in ${ROWS:-125000000 500000000}; do
  for P in ${PATHS:-sorted atomic}; do
    echo "== rows=$R path=$P"
    DQ_FREQ_PATH=$P timeout -k 10 ${TL:-150} python -u bench.py --workload c4 --c4-rows $R --steps 1 --warmup 1 \
      > $OUT/c4probe_${R}_$P.log 2>&1
    st=$?; tail -c 600 $OUT/c4probe_${R}_$P.log; echo
    if [ $st -ne 0 ]; then echo "STOP (exit $st)"; exit $st; fi
  done
done
echo ALL DONE
