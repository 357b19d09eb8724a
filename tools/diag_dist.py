"""Diagnostic: sharded dense solve variants, each in its own process (development aid)."""
import faulthandler, os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()

def one(heaps, ranks, graph):
    import numpy as np
    from gamesmanmpi_amd import Context, _lib
    ctx = Context(5, (heaps,), device=0)
    ctx.set_option(_lib.OPT_GRAPH, graph)
    ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
    print("solving", heaps, ranks, graph, flush=True)
    n, rec = ctx.solve(ctx.initial())
    print("solved", n, hex(rec), flush=True)
    n, rec = ctx.solve(ctx.initial())
    print("solved again", n, hex(rec), ctx.digest(), flush=True)

if __name__ == "__main__":
    if len(sys.argv) > 1:
        one(*map(int, sys.argv[1:4]))
    else:
        for args in [(4, 2, 0), (4, 2, 1), (6, 8, 0), (6, 8, 1)]:
            r = subprocess.run([sys.executable, __file__] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
            print(args, "rc", r.returncode, r.stdout.strip().replace("\n", " | "), r.stderr.strip()[-600:], flush=True)
