"""Per-workgroup trace of the row-dataflow kernel (GM_OPT_SUB_INTERLEAVE 13; needs the
GM_WK_TRACE build): t_start, t_loads_folded, t_children_ready, t_end, ids (development aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GM_TRACE_OUT", "gpurun_out/rf_trace.bin")
from gamesmanmpi_amd import Context, _lib
ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
ctx.set_option(_lib.OPT_SUB_INTERLEAVE, 13)
for i in range(3):
    ctx.solve(0xFFFFFFFF)
print("ok", os.path.getsize(os.environ["GM_TRACE_OUT"]))
