#!/usr/bin/env python3
"""Per-tier timeline of one dataflow box launch (development aid for csrc/dense_box.hip).

Needs a library built with -DGM_BOX_FLOW_TRACE=1 (tools/build_variant.sh ftr dense_box
-DGM_BOX_FLOW_TRACE=1); run a solve with GM_LIB_PATH set to it and
GM_BOX_FLOW_TRACE_OUT=<file>, then

    python tools/flow_trace.py <file>

Each group's record holds five s_memrealtime stamps (100 MHz): picked, children ready,
folded (child loads back and folded into LDS), walked, flagged (stores drained, flags
stored), and its first box id.  Prints, per box tier: groups, the first pick and the last
flag (µs from the launch's first pick), and the medians of wait, fold, walk and store.
The handoff column is the tier's first "ready" minus the tier before's last "flagged" --
how long a finished child box takes to be seen, at the chain's tightest point.
"""
import sys

import numpy as np


def tier_of(box):
    box = box.astype(np.int64)
    t = np.zeros_like(box)
    for i in range(4):
        t += (box >> (2 * i)) & 3
    for j in range(4):
        t += (box >> (8 + 3 * j)) & 7
    return t


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 6)
    ts = a[:, :5].astype(np.int64)
    t0 = ts[:, 0].min()
    us = (ts - t0) / 100.0
    tier = tier_of(a[:, 5] & 0xFFFFFFFF)
    print("groups %d, span %.1f us (first pick to last flag)" % (len(a), us[:, 4].max()))
    print("tier groups  first_pick  first_ready  last_flag   wait   fold   walk  store  handoff  (us)")
    prev_last = None
    for t in range(int(tier.max()) + 1):
        m = tier == t
        if not m.any():
            continue
        u = us[m]
        d = np.diff(u, axis=1)
        first_ready = u[:, 1].min()
        hand = first_ready - prev_last if prev_last is not None else float("nan")
        print("%4d %6d  %10.1f  %11.1f  %9.1f  %5.2f  %5.2f  %5.2f  %5.2f  %7.2f" % (
            t, m.sum(), u[:, 0].min(), first_ready, u[:, 4].max(), np.median(d[:, 0]), np.median(d[:, 1]),
            np.median(d[:, 2]), np.median(d[:, 3]), hand))
        prev_last = u[:, 4].max()
    d = np.diff(us, axis=1)
    print("all: median wait %.2f fold %.2f walk %.2f store %.2f us; summed wait %.1f us-groups" % (
        np.median(d[:, 0]), np.median(d[:, 1]), np.median(d[:, 2]), np.median(d[:, 3]), d[:, 0].sum()))


if __name__ == "__main__":
    main()
