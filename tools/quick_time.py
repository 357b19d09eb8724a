"""Quick timing of the dense 2^32 subtract solve across kernel variants (development aid)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib
variants = [(3, 256, 4), (3, 128, 1), (3, 256, 1)]
if len(sys.argv) > 1:
    variants = [tuple(int(x) for x in v.split(",")) for v in sys.argv[1:]]
ref = None
for v in variants:
    low, nt, x4 = v[:3]
    order = v[3] if len(v) > 3 else 1
    ctx = Context(5, (8,), device=0)
    ctx.set_option(_lib.OPT_SUB_LOW, low)
    ctx.set_option(_lib.OPT_SUB_THREADS, nt)
    ctx.set_option(_lib.OPT_SUB_INTERLEAVE, x4)
    ctx.set_option(_lib.OPT_SUB_ORDER, order)
    ts = []
    for i in range(5):
        t = time.perf_counter(); n, rec = ctx.solve(0xFFFFFFFF); ts.append(time.perf_counter() - t)
    d = ctx.digest()
    ref = ref or d
    print("low=%d nt=%d x4=%d order=%d best=%.2f ms med=%.2f ms pos/s=%.3e digest_ok=%s" % (
        low, nt, x4, order, min(ts) * 1e3, sorted(ts)[2] * 1e3, n / min(ts), d == ref), flush=True)
    ctx.close()
