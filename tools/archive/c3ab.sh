#!/bin/bash
# Same-box A/B of the utf8 HLL path (HLL kernel vs string pass) on C3's string variant.
mkdir -p gpurun_out
for i in 1 2; do
  for k in 0 1; do
    DQ_STRING_PASS_HLL=$k timeout -k 10 300 python -u bench.py --workload c3 --c3-type utf8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3ab_${k}_$i.log 2>&1 || exit $?
    echo "knob $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3ab_${k}_$i.log)"
  done
done
