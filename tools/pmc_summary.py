#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-trace / PMC CSVs of a bench run into profiles/.

    python tools/pmc_summary.py --kt gpurun_out/prof_kt --fetch gpurun_out/prof_fetch \
        --write gpurun_out/prof_write --kernel sub_tier_kernel_ --launches-per-solve 76 \
        --tag r01_subtract8 [--traffic-json profiles/traffic_subtract8.json]

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB,
collected in separate --pmc passes, and on gfx950 FETCH_SIZE reports half the bytes
of 16-B-per-lane streaming reads, so it is doubled (the tier kernel's reads are all
global_load_dwordx4 whole-block streams).
"""
import argparse
import collections
import csv
import json
import os
import shutil


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--launches-per-solve", type=int, required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--traffic-json")
    ap.add_argument("--algo-bytes-per-solve", type=float, default=None)
    a = ap.parse_args()
    os.makedirs("profiles", exist_ok=True)
    shutil.copy(os.path.join(a.kt, "run_kernel_stats.csv"), "profiles/%s_kernel_stats.csv" % a.tag)
    kt = [r for r in rows(os.path.join(a.kt, "run_kernel_trace.csv")) if a.kernel in r["Kernel_Name"]]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt]
    names = sorted(set(r["Kernel_Name"] for r in kt))
    out = {"kernel": names[0] if len(names) == 1 else names or a.kernel, "dispatches": len(durs),
           "avg_duration_us": sum(durs) / len(durs) / 1e3 if durs else None,
           "solve_kernel_ms": sum(durs) / (len(durs) / a.launches_per_solve) / 1e6 if durs else None,
           "launches_per_solve": a.launches_per_solve,
           "vgpr": sorted(set(r.get("VGPR_Count") for r in kt)), "lds_bytes": sorted(set(r.get("LDS_Block_Size") for r in kt))}
    pmc = {}
    for name, d in (("FETCH_SIZE", a.fetch), ("WRITE_SIZE", a.write)):
        if not d:
            continue
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(d, "run_counter_collection.csv"))
                if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
        if vals:
            pmc[name] = {"dispatches": len(vals), "kib_per_solve": sum(vals) / (len(vals) / a.launches_per_solve)}
            shutil.copy(os.path.join(d, "run_counter_collection.csv"), "profiles/%s_%s.csv" % (a.tag, name.lower()))
    out["pmc"] = pmc
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"]["kib_per_solve"] * 1024 * 2      # gfx950 half-count correction
        write = pmc["WRITE_SIZE"]["kib_per_solve"] * 1024
        out["hbm_read_bytes_per_solve"] = fetch
        out["hbm_write_bytes_per_solve"] = write
        out["hbm_bytes_per_solve"] = fetch + write
        out["hbm_bytes_per_launch"] = (fetch + write) / a.launches_per_solve
        if out["solve_kernel_ms"]:
            out["hbm_gbs"] = (fetch + write) / (out["solve_kernel_ms"] / 1e3) / 1e9
        if a.algo_bytes_per_solve:
            out["algo_bytes_per_solve"] = a.algo_bytes_per_solve
            out["algo_bytes_per_launch"] = a.algo_bytes_per_solve / a.launches_per_solve
        out["correction"] = "FETCH_SIZE x2 (gfx950, 16-B/lane streaming reads), KiB -> bytes"
    with open("profiles/%s_summary.json" % a.tag, "w") as f:
        json.dump(out, f, indent=1)
    if a.traffic_json and "hbm_bytes_per_launch" in out:
        with open(a.traffic_json, "w") as f:
            json.dump({"hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
                       "hbm_bytes_per_solve": out["hbm_bytes_per_solve"],
                       "source": "profiles/%s_summary.json" % a.tag}, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
