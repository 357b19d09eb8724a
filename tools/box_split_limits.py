#!/usr/bin/env python3
"""Tier-level limits of the halves split (development aid).

    python tools/box_split_limits.py [--rate 169] [--one-gpu-ms 3.24]

For G = 2, 4, 8 and the default plan (gm_box_plan, no GPU): every rank's groups per box-tier;
a rank's tier t starts when its own tier t - 1 and its lower neighbours' tier t - 1 are done
(+ a hop latency), and lasts groups / rate (the one-GPU thick-tier throughput, groups per us),
at least `floor` us per launch.  Prints the makespan and the speedup over the one-GPU time:
with no floor and no latency it is the limit any tier-ordered schedule of this partition can
reach -- the upper ranks' work sits in later tiers (stagger)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=169.0)
    ap.add_argument("--one-gpu-ms", type=float, default=3.24)
    a = ap.parse_args()
    for G in (2, 4, 8):
        g = G.bit_length() - 1
        groups = [(np.diff(_lib.box_plan(G, r, _lib.BOXPLAN_TIER_OFF).astype(np.int64)) + 1) // 2 for r in range(G)]
        T = len(groups[0])
        for lat, floor in ((0.0, 0.0), (5.0, 0.0), (20.0, 8.0)):
            end = np.zeros((G, T))
            for t in range(T):
                for r in range(G):
                    st = end[r, t - 1] if t else 0.0
                    for ax in range(g):
                        if (r >> ax) & 1 and t:
                            st = max(st, end[r ^ (1 << ax), t - 1] + lat)
                    n = groups[r][t]
                    end[r, t] = st + (max(n / a.rate, floor) if n else 0.0)
            ms = end[:, -1].max() / 1000
            print(json.dumps({"ranks": G, "hop_latency_us": lat, "launch_floor_us": floor, "makespan_ms": round(ms, 4),
                              "speedup": round(a.one_gpu_ms / ms, 3)}))


if __name__ == "__main__":
    main()
