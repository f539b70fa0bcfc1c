#!/bin/bash
set -u
LIBS="s0 s1 s2 s3 s4" WL=c4 bash tools/kprof_ab.sh 2>&1 | grep -E "ms_per_step|stage_part|STOP|FAILED"
