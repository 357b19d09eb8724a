"""Time dense solves of the 8-heap subtraction game from roots whose box is a fraction of
the 2^32 table (development aid): does a smaller working set per tier launch (the
producer tiers fitting the 256 MiB Infinity Cache) raise the rate per position?

    python tools/box_time.py [root ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib  # noqa: E402


def main():
    roots = [int(r, 16) for r in sys.argv[1:]] or [0xFFFFFFFF, 0x7FFFFFFF, 0x77FFFFFF, 0x777FFFFF, 0x3FFFFFFF,
                                                  0xFFFFFFF7, 0xFFFFF777]
    for root in roots:
        ctx = Context(_lib.GAME_SUBTRACT, (8,), device=0)
        ctx.set_option(_lib.OPT_TIMING, 1)
        ctx.solve(root)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            n, rec = ctx.solve(root)
            ts.append(time.perf_counter() - t)
        st = ctx.stats()
        m = sorted(ts)[2]
        print("root %#010x: %11d positions, %3d launches, median %.3f ms, kernel %.3f ms, %.3e positions/s"
              % (root, n, st["kernel_launches"], m * 1e3, st["kernel_ms"], n / m), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
