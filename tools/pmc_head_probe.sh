#!/bin/bash
# SQ counters of the head probe's kernels (instruction mix, issue activity, waits): two passes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_head_probe}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS -d $OUT/a -o run --output-format csv -- python3 tools/probe/head_probe.py 3 > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- python3 tools/probe/head_probe.py 3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
python3 - <<PY
import csv, glob, collections
for pas in ("a", "b"):
    f = glob.glob("$OUT/" + pas + "/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"]
    fam = collections.defaultdict(list)
    for d, cs in per.items():
        n = names[d].replace("(anonymous namespace)::", "").split("(")[0][:60]
        fam[n].append(cs)
    for n, l in fam.items():
        if "head" not in n: continue
        avg = {k: sum(c[k] for c in l) / len(l) for k in l[0]}
        print(pas, n, {k: "%.3g" % v for k, v in sorted(avg.items())})
PY
