#!/bin/bash
# HBM traffic per step of one bench workload from PMC counters (MI355X_MICROARCH.md §HBM):
# one rocprofv3 --pmc pass per counter (no tracing combined with --pmc); on gfx950 FETCH_SIZE
# reports 1/2 of a wide streaming read, so read bytes = 2 * FETCH_SIZE(KiB) * 1024, write
# bytes = WRITE_SIZE(KiB) * 1024.  Sums the dispatches of every kernel matching KERNEL (a
# regex) over the profiled steps and divides by the step count (warmup 1 + STEPS timed).
#   WL=c4 KERNEL='dq::' STEPS=1 TAG=r02 bash tools/pmc_traffic.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r02}
WL=${WL:-c2}
STEPS=${STEPS:-1}
for C in FETCH_SIZE WRITE_SIZE; do
  D="$OUT/pmct_${WL}_${C}_$TAG"
  timeout -s KILL ${TL:-240} rocprofv3 --pmc $C --output-format csv -d "$D" -o run \
    -- python -u bench.py --workload $WL --steps $STEPS --warmup 1 --no-cpu-baseline --no-side-passes ${BENCH_ARGS:-} > "$D.log" 2>&1
  st=$?
  if [ $st -ne 0 ]; then echo "STOP: pmc $C exit $st"; tail -5 "$D.log"; exit $st; fi
done
python - <<PY
import csv, glob, json, re, collections, sys
sys.path.insert(0, ".")
import bench
pat = re.compile(r"""$KERNEL""")
out = {"workload": "$WL", "kernel_regex": r"""$KERNEL""", "steps_profiled": $STEPS + 1,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each; read = 2 x FETCH_SIZE (gfx950)",
       "kernel_src_digest": bench.kernel_source_digest(), "commit": "${COMMIT:-unknown}",
       "bench_args": "${BENCH_ARGS:-}"}
per_kernel = collections.defaultdict(lambda: {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "dispatches": set()})
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob("$OUT/pmct_${WL}_%s_$TAG/**/*counter_collection.csv" % c, recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if row.get("Counter_Name") == c and pat.search(name):
                k = per_kernel[name.split("(")[0]]
                k[c] += float(row["Counter_Value"])
                k["dispatches"].add(row["Dispatch_Id"])
n = $STEPS + 1
tot_r = tot_w = 0.0
ks = {}
for name, k in per_kernel.items():
    r = 2.0 * 1024 * k["FETCH_SIZE"] / n
    w = 1024 * k["WRITE_SIZE"] / n
    tot_r += r
    tot_w += w
    ks[name] = {"read_bytes_per_step": r, "write_bytes_per_step": w, "dispatches": len(k["dispatches"])}
out["kernels"] = ks
out["hbm_read_bytes_per_step"] = tot_r
out["hbm_write_bytes_per_step"] = tot_w
out["hbm_bytes_per_step"] = tot_r + tot_w
json.dump(out, open("$OUT/traffic_${WL}_$TAG.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))
PY
