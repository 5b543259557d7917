"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md § HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE come from separate passes (TCC slots); on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads, so it is doubled; both are in KiB.

usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [kernel-substr]
       [exclude-substr] [steps]
kernel-substr may list alternatives separated by '|' (e.g. "gemm_kernel|wgrad_conv3_kernel|gemm_reduce_kernel": every
kernel one aw_gemm / aw_gemm_grouped call can launch); exclude-substr (e.g. "<float") leaves the exact-f32
instantiations out of a bf16 family; with the number of traced steps the family's bytes per step are added.
Prints per-kernel average bytes per launch (and the family aggregate) as JSON."""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            per[name].append(float(row["Counter_Value"]))
    return per


def main(fetch_csv, write_csv, sub="gemm_kernel", exclude=None, steps=None):
    subs = sub.split("|")
    exclude = exclude or None
    fe = load(fetch_csv, "FETCH_SIZE")
    wr = load(write_csv, "WRITE_SIZE")
    out = {}
    tot_b, tot_n = 0.0, 0
    for name in sorted(set(fe) | set(wr)):
        f = fe.get(name, [])
        w = wr.get(name, [])
        if not f or not w:
            continue
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        out[name[:120]] = {"launches": len(f), "fetch_bytes": fb, "write_bytes": wb, "bytes_per_launch": fb + wb}
        if any(x in name for x in subs) and not (exclude and exclude in name):
            tot_b += (fb + wb) * len(f)
            tot_n += len(f)
    res = {"family": sub, "excluded": exclude, "launches": tot_n, "avg_bytes_per_launch": tot_b / tot_n if tot_n else None}
    if steps:
        res["steps"] = int(steps)
        res["bytes_per_step"] = tot_b / int(steps)
    res["kernels"] = out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
