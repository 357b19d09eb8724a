"""Per-rank solo time (GM_OPT_DIST_SOLO: one rank's tier launches alone, results invalid) of
the sharded dense solve for tier-kernel variants (GM_OPT_SUB_INTERLEAVE 6 = b4, 8 = one wave
per group) at 2, 4, 8 loopback ranks (development aid).

    python tools/solo_variants.py [heaps]
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
        for variant in [int(v) for v in os.environ.get("GM_SOLO_VARIANTS", "6").split(",")]:
            ctx = Context(_lib.GAME_SUBTRACT, (heaps,), device=0)
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, G)
            ctx.set_option(_lib.OPT_SUB_INTERLEAVE, variant)
            root = ctx.initial()
            solo = []
            for r in range(G):
                ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)
                solo.append(timed(ctx, root))
            ctx.set_option(_lib.OPT_DIST_SOLO, 0)
            full = timed(ctx, root)
            print("G=%d variant=%d solo max %.2f ms (ranks %s) loopback whole %.2f ms"
                  % (G, variant, max(solo), " ".join("%.2f" % x for x in solo), full), flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
