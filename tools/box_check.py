"""Box engine (GM_OPT_SUB_INTERLEAVE 20) check on the GPU: the 2^32 table's digest against
the committed C-oracle digest, custom roots against the block engine, and solve times."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib  # noqa: E402

SUB = 5
REF = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "oracle_digests.json")))["subtract_8"]


def solve(root, variant, reps=1, **opts):
    ctx = Context(SUB, (8,), device=0)
    ctx.set_option(_lib.OPT_SUB_INTERLEAVE, variant)
    ctx.set_option(_lib.OPT_TIMING, 1)
    for k, v in opts.items():
        ctx.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    ts = []
    for _ in range(reps):
        n, rec = ctx.solve(root)
        ts.append(ctx.stats()["kernel_ms"])
    return ctx, n, rec, ts


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    ok = True
    if which in ("all", "full"):
        ctx, n, rec, ts = solve(0xFFFFFFFF, 20, reps=int(os.environ.get("REPS", "10")))
        dg = ctx.digest()
        good = (n, rec) == (REF["positions"], REF["root_record"]) and dg == (REF["digest"], REF["positions"])
        ok &= good
        print("box full: n=%d rec=%d digest=%d ok=%s kernel_ms=%s" % (n, rec, dg[0], good, ["%.3f" % t for t in ts]), flush=True)
        ctx.close()
    if which in ("all", "roots"):
        for root in (0x7, 0x12345678, 0xFF00FF00, 0x0000FFFF, 0xFFFF0000, 0x33333333, 0x9ABCDEF1, 0xF0F0F0F0):
            a, n1, r1, _ = solve(root, 20)
            da = a.digest()
            a.close()
            b, n2, r2, _ = solve(root, 10)
            db = b.digest()
            b.close()
            good = (n1, r1, da) == (n2, r2, db)
            ok &= good
            print("root 0x%08x: box %s block %s ok=%s" % (root, (n1, r1, da), (n2, r2, db), good), flush=True)
    print("ALL OK" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
