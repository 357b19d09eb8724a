"""Per-kernel sums of rocprofv3 --pmc counter CSVs (several passes) -> one JSON.

    python tools/pmc_kernels.py OUT.json DIR [DIR ...] [--solves N]

Each DIR holds a run_counter_collection.csv of one --pmc pass.  Values are summed
per (kernel base name, counter) and divided by --solves.  FETCH_SIZE / WRITE_SIZE
are KiB; FETCH_SIZE is reported raw and doubled (the gfx950 correction for 16-B
per-lane streaming reads, MI355X_MICROARCH.md 'HBM'; random 8-16-B accesses are
uncalibrated, so both are kept).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    args = sys.argv[1:]
    solves = 1
    if "--solves" in args:
        i = args.index("--solves")
        solves = int(args[i + 1])
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"(\w+_kernel\w*)", r["Kernel_Name"])
                name = m.group(1) if m else r["Kernel_Name"].split("(")[0]
                agg[name][r["Counter_Name"]] += float(r["Counter_Value"]) / solves
    res = {}
    for k, cs in agg.items():
        e = dict(cs)
        if "FETCH_SIZE" in e:
            e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in e:
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
        if "SQ_LDS_BANK_CONFLICT" in e and e.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_ratio"] = e["SQ_LDS_BANK_CONFLICT"] / e["SQ_LDS_IDX_ACTIVE"]
        if e.get("TCC_HIT_sum") is not None and e.get("TCC_MISS_sum") is not None:
            e["tcc_hit_rate"] = e["TCC_HIT_sum"] / max(1.0, e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        res[k] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
