import os, sys
sys.path.insert(0, "/root/repo")
from gamesmanmpi_amd import Context, _lib
ctx = Context(5, (8,), device=0)
ctx.set_option(_lib.OPT_TIMING, 1)
for _ in range(4):
    n, rec = ctx.solve(0xFFFFFFFF)
    print("kernel_ms", ctx.stats()["kernel_ms"], flush=True)
