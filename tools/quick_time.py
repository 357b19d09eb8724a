"""Quick timing of the dense 2^32 subtract solve (development aid)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib
for low in (3, 2):
    ctx = Context(5, (8,), device=0)
    ctx.set_option(_lib.OPT_SUB_LOW, low)
    for graph in (0, 1):
        ctx.set_option(_lib.OPT_GRAPH, graph)
        for timing in (0, 1):
            ctx.set_option(_lib.OPT_TIMING, timing)
            ts = []
            for i in range(4):
                t = time.perf_counter(); n, rec = ctx.solve(0xFFFFFFFF); ts.append(time.perf_counter() - t)
            st = ctx.stats()
            print("low=%d graph=%d timing=%d n=%d rec=%#x best=%.2f ms med=%.2f ms kernel_ms=%.2f launches=%d pos/s=%.3e" % (
                low, graph, timing, n, rec, min(ts)*1e3, sorted(ts)[2]*1e3, st['kernel_ms'], st['kernel_launches'], n/min(ts)), flush=True)
    ctx.close()
