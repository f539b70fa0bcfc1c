#!/bin/bash
# PMC counters of one kernel of one bench workload, one rocprofv3 --pmc pass per counter group
# (no tracing combined with --pmc).  Usage:
#   WL=c3 KERNEL=dq_hll_kernel PASSES="SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVES,GRBM_GUI_ACTIVE;FETCH_SIZE" \
#     BENCH_ARGS="--c3-rows 125000000" TAG=r01 bash tools/pmc_kernel.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r01}
IFS=';' read -ra GROUPS_ <<< "$PASSES"
k=0
for G in "${GROUPS_[@]}"; do
  C=$(echo "$G" | tr ',' ' ')
  D="$OUT/pmck_${WL}_${TAG}_$k"
  timeout -s KILL ${TL:-180} rocprofv3 --pmc $C --output-format csv -d "$D" -o run \
    -- python -u bench.py --workload $WL --steps 1 --warmup 1 --no-cpu-baseline --no-side-passes ${BENCH_ARGS:-} > "$D.log" 2>&1
  st=$?
  if [ $st -ne 0 ]; then echo "STOP: pmc pass '$G' exit $st"; tail -5 "$D.log"; exit $st; fi
  k=$((k + 1))
done
python - <<PY
import csv, glob, json, collections
res = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("$OUT/pmck_${WL}_${TAG}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "$KERNEL" in row.get("Kernel_Name", ""):
            res[row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
out = {c: [v for _, v in sorted(d.items())] for c, d in res.items()}
json.dump({"workload": "$WL", "kernel": "$KERNEL", "per_dispatch": out}, open("$OUT/pmck_${WL}_$TAG.json", "w"), indent=1)
print(json.dumps(out))
PY
