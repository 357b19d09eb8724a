"""Box-engine solve time with the library's own table vs a torch-allocated (adopted) table,
and with the library's stream vs a torch stream (bench.py's setting)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from gamesmanmpi_amd import Context, _lib  # noqa: E402


def run(label, adopt=False, tstream=False, offset=0):
    ctx = Context(5, (8,), device=0)
    ctx.set_option(_lib.OPT_TIMING, 1)
    keep = None
    if adopt:
        keep = torch.empty((1 << 32) + offset, dtype=torch.uint8, device="cuda")
        ctx.adopt_dense_table(keep.data_ptr() + offset, 1 << 32)
    if tstream:
        s = torch.cuda.Stream()
        torch.cuda.set_stream(s)
        ctx.set_stream(s.cuda_stream)
    ts = []
    for _ in range(8):
        ctx.solve(0xFFFFFFFF)
        ts.append(ctx.stats()["kernel_ms"])
    d = ctx.digest()
    print("%-34s median %.3f ms  min %.3f  digest %#x  ptr %#x" % (label, statistics.median(ts[2:]), min(ts[2:]), d[0],
                                                               keep.data_ptr() if keep is not None else 0), flush=True)
    ctx.close()
    del keep
    torch.cuda.empty_cache()


run("own table, own stream")
run("torch table, own stream", adopt=True)
run("torch table, torch stream", adopt=True, tstream=True)
run("own table, torch stream", tstream=True)
run("torch table +4096 offset", adopt=True, offset=4096)
