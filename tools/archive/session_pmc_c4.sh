#!/bin/bash
set -u
WL=c4 KERNEL=dq_freq_stage_part_kernel TAG=r03s PASSES="SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES,GRBM_GUI_ACTIVE;SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY" bash tools/pmc_kernel.sh || exit $?
python3 - <<'PY'
import csv, glob, collections, json
for kern in ("dq_freq_stage_part_kernel", "dq_freq_part_kernel", "dq_freq_agg_packed_kernel"):
    res = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob("gpurun_out/pmck_c4_r03s_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row.get("Kernel_Name", ""):
                res[row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    avg = {c: sum(d.values()) / len(d) for c, d in res.items()}
    print(kern, json.dumps({k: round(v / 1e6, 2) for k, v in sorted(avg.items())}))
    json.dump({"kernel": kern, "avg_per_dispatch": avg}, open("gpurun_out/pmc_c4_%s_r03s.json" % kern, "w"), indent=1)
PY
find gpurun_out -path "*pmck_c4_r03s_*" -name "*counter_collection.csv" -delete
