#!/usr/bin/env python3
"""Per-box-tier times of the one-GPU 2^32 solve from a rocprofv3 kernel trace.

    python tools/box_tier_trace.py <trace dir> [--json out.json]

The trace is of `bench.py` (one GPU, box engine): every solve is 41 launches of
box_tier_kernel<false>, box-tier 0 first.  Per box-tier: its groups (two boxes each: the boxes
of the 4x4x4x4x2x2x2x2 lattice whose coordinates sum to the tier), the median launch duration
over the traced solves, and what the tier would take at the throughput of the thick tiers
(groups / (groups per us of the tiers with >= 2 resident rounds)).  A thin tier (fewer groups
than one resident round of 2,048) pays for its latency chain; the sum of (duration - time at
throughput) over them is all that any thin-tier scheme could save at N = 1.
"""
import argparse
import csv
import glob
import json

import numpy as np


def tier_groups():
    b = np.arange(1 << 20)
    t = sum((b >> (2 * i)) & 3 for i in range(4)) + sum((b >> (8 + 3 * j)) & 7 for j in range(4))
    n = np.bincount(t, minlength=41)
    return (n + 1) // 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--json", default=None)
    ap.add_argument("--round", type=int, default=2048, help="groups per resident round")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(a.trace + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "box_tier_kernel<false" in r["Kernel_Name"] or "box_tier4_kernel<false" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    n = len(rows) // 41
    if n == 0:
        raise SystemExit("no complete solve in the trace")
    rows = rows[-41 * n:]
    dur = np.array([(e - s) / 1e3 for s, e in rows]).reshape(n, 41)        # us
    span = np.array([(rows[41 * i + 40][1] - rows[41 * i][0]) / 1e3 for i in range(n)])
    med = np.median(dur, axis=0)
    g = tier_groups()
    thick = g >= 2 * a.round
    rate = g[thick].sum() / med[thick].sum()                                # groups per us
    ideal = g / rate
    thin = g < a.round
    excess = np.maximum(0.0, med - ideal)
    out = {"solves": int(n), "solve_span_us_median": float(np.median(span)),
           "launch_sum_us_median": float(np.median(dur.sum(axis=1))),
           "thick_tier_rate_groups_per_us": float(rate),
           "thin_tiers": [int(t) for t in np.nonzero(thin)[0]],
           "thin_tier_us": float(med[thin].sum()), "thin_tier_us_at_throughput": float(ideal[thin].sum()),
           "thin_tier_excess_us": float(excess[thin].sum()),
           "tiers": [{"tier": t, "groups": int(g[t]), "us": round(float(med[t]), 2),
                      "us_at_throughput": round(float(ideal[t]), 2)} for t in range(41)]}
    print("tier  groups      us   at-throughput")
    for t in range(41):
        print("%4d %7d %8.2f %8.2f%s" % (t, g[t], med[t], ideal[t], "  thin" if thin[t] else ""))
    print("solves %d: span %.1f us (median), launch sum %.1f us; thick-tier rate %.1f groups/us" %
          (n, out["solve_span_us_median"], out["launch_sum_us_median"], rate))
    print("thin tiers (%d): %.1f us, %.1f us at throughput, excess %.1f us = %.1f %% of the span" %
          (thin.sum(), out["thin_tier_us"], out["thin_tier_us_at_throughput"], out["thin_tier_excess_us"],
           100 * out["thin_tier_excess_us"] / out["solve_span_us_median"]))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
