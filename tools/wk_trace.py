"""Per-workgroup phase trace of the dense walker kernel (development aid).

Needs the diagnostic build (tools/build_exp.sh "tr=-DGM_WK_TRACE", GM_LIB_PATH=_exp/libgm_tr.so);
writes GM_TRACE_OUT (default gpurun_out/wk_trace.bin) for the last of a few solves:
8 u64 per workgroup: t_start, t_passA_done, t_walk_done, t_stores_issued (s_memrealtime,
100 MHz), HW_ID | XCC_ID << 32, blockIdx | hp0 << 32, t_loads_back, t_folds_written.
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GM_TRACE_OUT", "gpurun_out/wk_trace.bin")
from gamesmanmpi_amd import Context, _lib
ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
for i in range(4):
    t = time.perf_counter(); n, rec = ctx.solve(0xFFFFFFFF); dt = time.perf_counter() - t
    print("solve %d: %.2f ms" % (i, dt * 1e3), flush=True)
print("trace bytes", os.path.getsize(os.environ["GM_TRACE_OUT"]))
