#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per access shape (traffic_probe.hip): one rocprofv3 --pmc pass per
# counter over the probe binary, joined with the bytes each probe moves by construction.
# Writes gpurun_out/traffic_probe.json: per probe counter KiB, algorithmic bytes and the ratio.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/traffic_probe > gpurun_out/traffic_probe_bytes.jsonl || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/tprobe_$C -o run -- ./tools/ubench/traffic_probe \
    > gpurun_out/tprobe_$C.log 2>&1 || { echo "STOP pmc $C"; tail -5 gpurun_out/tprobe_$C.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
want = {}
for ln in open("gpurun_out/traffic_probe_bytes.jsonl"):
    if ln.startswith("{"):
        d = json.loads(ln)
        want[d.get("kname", d["kernel"])] = d
got = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob("gpurun_out/tprobe_%s/**/*counter_collection.csv" % c, recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            k = k[5:] if k.startswith("void ") else k
            if row.get("Counter_Name") == c and k in want:
                got.setdefault(k, {}).setdefault(c, 0.0)
                got[k][c] += float(row["Counter_Value"])
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (KiB), one pass each, over tools/ubench/traffic_probe",
       "probes": {}}
for kn, d in want.items():
    g, k = got.get(kn, {}), d["kernel"]
    fr, wr = g.get("FETCH_SIZE", 0.0) * 1024, g.get("WRITE_SIZE", 0.0) * 1024
    out["probes"][k] = {"shape": d["shape"], "read_bytes": d["read_bytes"], "write_bytes": d["write_bytes"],
                        "fetch_size_bytes": fr, "write_size_bytes": wr,
                        "fetch_over_read": fr / d["read_bytes"] if d["read_bytes"] else None,
                        "write_over_written": wr / d["write_bytes"] if d["write_bytes"] else None}
json.dump(out, open("gpurun_out/traffic_probe.json", "w"), indent=1)
for k, v in out["probes"].items():
    print("%-26s fetch/read %s  write/written %s" % (k, v["fetch_over_read"] and "%.3f" % v["fetch_over_read"],
                                                    v["write_over_written"] and "%.3f" % v["write_over_written"]))
PY
find gpurun_out -path "*tprobe_*" -name "*.csv" -size +5M -delete
