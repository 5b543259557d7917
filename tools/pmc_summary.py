"""Per-kernel-family summary of one tools/prof_round.sh directory: average duration (kernel trace), HBM bytes per
launch (FETCH_SIZE x 2 per the gfx950 note in MI355X_MICROARCH.md, + WRITE_SIZE; both KiB), achieved HBM GB/s,
MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the SIMD-cycles of the launch: GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs), wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES) and the LDS
bank-conflict rate (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def family(name):
    """Kernel name without its argument list (and without the '(anonymous namespace)::' qualifier, whose own
    parenthesis would otherwise cut the whole name)."""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:140]


def one(path_glob):
    files = glob.glob(path_glob)
    return files[0] if files else None


def counters(path):
    per = defaultdict(lambda: defaultdict(float))     # (dispatch) -> counter -> value (summed over dims)
    names = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    fam = defaultdict(list)
    for d, cs in per.items():
        fam[family(names[d])].append(cs)
    return fam


def main(d, out=None):
    trace = one(os.path.join(d, "trace", "*kernel_trace.csv")) or one(os.path.join(d, "trace", "*", "*kernel_trace.csv"))
    dur = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        dur[family(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    sq = counters(one(os.path.join(d, "pmc_sq", "*counter_collection.csv")))
    fe = counters(one(os.path.join(d, "pmc_fetch", "*counter_collection.csv")))
    wr = counters(one(os.path.join(d, "pmc_write", "*counter_collection.csv")))
    res = {}
    for f, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        avg_ns = sum(ds) / len(ds)
        e = {"launches": len(ds), "total_ms": round(sum(ds) / 1e6, 3), "avg_us": round(avg_ns / 1e3, 2)}
        if f in fe and f in wr:
            fb = 2.0 * 1024.0 * sum(c["FETCH_SIZE"] for c in fe[f]) / len(fe[f])
            wb = 1024.0 * sum(c["WRITE_SIZE"] for c in wr[f]) / len(wr[f])
            e.update(hbm_bytes_per_launch=round(fb + wb), fetch_bytes=round(fb), write_bytes=round(wb),
                     hbm_gbs=round((fb + wb) / avg_ns, 1))
        if f in sq:
            cs = sq[f]
            tot = lambda k: sum(c.get(k, 0.0) for c in cs)  # noqa: E731
            cyc = tot("GRBM_GUI_ACTIVE") / XCDS
            if cyc > 0:
                e["mfma_busy_frac"] = round(tot("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * SIMDS), 4)
                e["clock_ghz"] = round(cyc / len(cs) / avg_ns, 3)
            wc = tot("SQ_WAVE_CYCLES")
            if wc > 0:
                e["wave_split"] = {k: round(tot(c) / wc, 3) for k, c in (("wait_any", "SQ_WAIT_ANY"),
                                                                       ("wait_inst", "SQ_WAIT_INST_ANY"),
                                                                       ("active", "SQ_ACTIVE_INST_ANY"))}
            li = tot("SQ_LDS_IDX_ACTIVE")
            if li > 0:
                e["lds_bank_conflict_rate"] = round(tot("SQ_LDS_BANK_CONFLICT") / li, 4)
        res[f] = e
    txt = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
