#!/bin/bash
set -u
LIBS="g0 a5 a1 a4 g0 a5" WL=c4 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|part_kernel|agg_packed|STOP|FAILED"
