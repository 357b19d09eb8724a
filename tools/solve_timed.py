"""Time repeated strong solves of one game through libgmsolve.so (development aid).

    python tools/solve_timed.py toot 6 4 [repeats] [virtual_ranks]
    python tools/solve_timed.py othello 4 4
    python tools/solve_timed.py subtract 8 [repeats] [virtual_ranks]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gamesmanmpi_amd import Context, _lib  # noqa: E402

GAMES = {"f2o": _lib.GAME_FOUR_TO_ONE, "ttt": _lib.GAME_TTT, "toot": _lib.GAME_TOOT,
         "othello": _lib.GAME_OTHELLO, "subtract": _lib.GAME_SUBTRACT}


def main():
    name = sys.argv[1]
    nparams = {"f2o": 0, "ttt": 0, "toot": 2, "othello": 2, "subtract": 1}[name]
    params = tuple(int(x) for x in sys.argv[2:2 + nparams])
    rest = sys.argv[2 + nparams:]
    repeats = int(rest[0]) if rest else 3
    vranks = int(rest[1]) if len(rest) > 1 else 1
    ctx = Context(GAMES[name], params, device=0)
    if vranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, vranks)
    for key, val in os.environ.items():
        if key.startswith("GM_OPT_"):
            ctx.set_option(getattr(_lib, key[3:]), int(val))
    root = ctx.initial()
    for i in range(repeats):
        t = time.perf_counter()
        n, rec = ctx.solve(root)
        dt = time.perf_counter() - t
        st = ctx.stats()
        print("%s %s solve %d: %d positions, root %#06x, %.1f ms (%.3e positions/s); forward %.1f ms, "
              "backward %.1f ms, exchanged %d B" % (name, params, i, n, rec, dt * 1e3, n / dt, st["forward_ms"],
                                                     st["backward_ms"], st["exchanged_bytes"]), flush=True)
    print("digest", ctx.digest(), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
