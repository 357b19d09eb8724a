"""Per-rank critical path of the sharded dense solve under both block-owner functions
(development aid): for G = 2, 4, 8 loopback ranks, GM_OPT_DIST_SOLO times each rank's
tier launches alone on the GPU (results invalid in that mode), then the whole loopback
solve.  The max over ranks of the solo time is the compute critical path of one
rank per GPU.

    python tools/owner_solo.py [heaps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib  # noqa: E402


def timed(ctx, root, reps=4):
    ctx.solve(root)
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        ctx.solve(root)
        best = min(best, time.perf_counter() - t)
    return best * 1e3


def main():
    heaps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    for G in (2, 4, 8):
        for owner in (0, 1):
            ctx = Context(_lib.GAME_SUBTRACT, (heaps,), device=0)
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, G)
            ctx.set_option(_lib.OPT_DIST_OWNER, owner)
            root = ctx.initial()
            solo = []
            for r in range(G):
                ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)
                solo.append(timed(ctx, root))
            ctx.set_option(_lib.OPT_DIST_SOLO, 0)
            full = timed(ctx, root)
            d = ctx.digest()
            print("G=%d owner=%d solo per rank ms %s max %.3f | loopback whole solve %.2f ms, exchanged %d B, "
                  "digest %s" % (G, owner, " ".join("%.3f" % x for x in solo), max(solo), full,
                                 ctx.stats()["exchanged_bytes"], d), flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
