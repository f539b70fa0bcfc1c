#!/bin/bash
# HBM traffic of the fused scan from PMC counters (separate passes, no tracing combined with
# --pmc), per MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a wide streaming read on
# gfx950, so bytes = 2 * FETCH_SIZE(KiB) * 1024; WRITE_SIZE is exact for 16-B stores.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r01}
ROWS=${ROWS:-1000000000}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$TAG" -o run \
    -- python -u bench.py --steps 2 --warmup 1 --rows $ROWS --no-cpu-baseline --no-side-passes > "$OUT/pmc_${C}_$TAG.log" 2>&1
  st=$?
  if [ $st -ne 0 ]; then echo "STOP: pmc $C exit $st"; tail -5 "$OUT/pmc_${C}_$TAG.log"; exit $st; fi
done
python - <<PY
import csv, glob, json, collections
out = {"rows": $ROWS, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, bench.py C2 workload"}
per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob("$OUT/pmc_%s_$TAG/**/*counter_collection.csv" % c, recursive=True)
    vals = collections.defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if "dq_scan_values_kernel" in name and row.get("Counter_Name") == c:
                vals[row.get("Dispatch_Id")].append(float(row["Counter_Value"]))
    per[c] = [sum(v) for _, v in sorted(vals.items(), key=lambda kv: int(kv[0]))]
    out[c + "_kib_per_dispatch"] = per[c]
# one consume = the int64 launch + the fp64 launch (consecutive dispatches)
f = per["FETCH_SIZE"]
w = per["WRITE_SIZE"]
pairs = [f[i] + f[i + 1] for i in range(0, len(f) - 1, 2)]
wpairs = [w[i] + w[i + 1] for i in range(0, len(w) - 1, 2)]
if pairs:
    read_b = 2.0 * 1024 * sorted(pairs)[len(pairs) // 2]
    write_b = 1024 * sorted(wpairs)[len(wpairs) // 2] if wpairs else 0.0
    out["hbm_read_bytes_per_launch"] = read_b
    out["hbm_write_bytes_per_launch"] = write_b
    out["hbm_bytes_per_launch"] = read_b + write_b
json.dump(out, open("$OUT/traffic_$TAG.json", "w"), indent=1)
print(json.dumps(out)[:600])
PY
