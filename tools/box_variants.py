"""Times box-engine build variants (tools/build_variant.sh libraries): one subprocess per
library, kernel_ms of 10 solves of the 2^32 game (ablation variants give invalid tables).
    python tools/box_variants.py _exp/libgm_a.so _exp/libgm_b.so ..."""
import os
import subprocess
import sys

CODE = r'''
import os, sys, statistics
sys.path.insert(0, %r)
from gamesmanmpi_amd import Context, _lib
ctx = Context(5, (8,), device=0)
ctx.set_option(_lib.OPT_SUB_INTERLEAVE, int(os.environ.get("VARIANT", "20")))
ctx.set_option(_lib.OPT_TIMING, 1)
ts = []
for _ in range(int(os.environ.get("SOLVES", "24"))):
    n, rec = ctx.solve(0xFFFFFFFF)
    ts.append(ctx.stats()["kernel_ms"])
d = ctx.digest()
print("%%-28s min %%.3f median %%.3f ms  rec %%d digest %%d" %% (os.path.basename(os.environ.get("GM_LIB_PATH", "default")), min(ts[2:]), statistics.median(ts[2:]), rec, d[0]), flush=True)
''' % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

for lib in sys.argv[1:]:
    env = dict(os.environ, GM_LIB_PATH=lib)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout.strip() or r.stderr.strip()[-500:], flush=True)
