#!/usr/bin/env python3
"""Per-rank GPU time of the sharded box solve (8-heap game, root 0xFFFFFFFF) on ONE GPU.

    python tools/box_shard_time.py [--ranks 1 2 4 8] [--reps 10]

Virtual ranks (GM_OPT_VIRTUAL_RANKS): every rank's tier launches run alone, one rank
after the other, each on its own table.  A rank of the sharded box solve never waits for
another (csrc/dense_box.hip box_plan: no exchange), so a rank's event span here is its
whole multi-GPU job; the max over ranks is the N-GPU solve's GPU time.  Prints, per G,
the median over reps of every rank's kernel ms, the max, the speedup against G = 1, and
the digest check against the committed oracle digest.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    from gamesmanmpi_amd import Context, _lib
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_digests.json")))["subtract_8"]
    stream = torch.cuda.Stream()
    base = None
    out = []
    for G in a.ranks:
        ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
        ctx.set_stream(stream.cuda_stream)
        ctx.set_option(_lib.OPT_TIMING, 1)
        if G > 1:
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, G)
        root = 0xFFFFFFFF
        ctx.solve(root)
        ms = []
        for _ in range(a.reps):
            ctx.solve(root)
            ms.append([r["kernel_ms"] for r in ctx.rank_stats()])
        ms = np.median(np.array(ms), axis=0)
        rs = ctx.rank_stats()
        d = ctx.digest()
        ok = d == (ref["digest"], ref["positions"])
        mx = float(ms.max())
        base = base or mx
        line = {"ranks": G, "per_rank_ms": [round(float(x), 4) for x in ms], "max_ms": round(mx, 4),
                "speedup_vs_1": round(base / mx, 3), "boxes_per_rank": rs[0]["boxes"], "ties_per_rank": rs[0]["ties"],
                "digest_ok": ok}
        print(json.dumps(line), flush=True)
        out.append(line)
        ctx.close()
        torch.cuda.empty_cache()
    return 0 if all(x["digest_ok"] for x in out) else 1


if __name__ == "__main__":
    sys.exit(main())
