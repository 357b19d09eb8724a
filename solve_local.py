#!/usr/bin/env python3
"""Drop-in for the reference's ``solve_local.py``: one process, one line of output.

    python solve_local.py GAME_FILE [--custom FILE --init_pos NAME] [--dims LxH] [--remoteness]

The reference (solve_local.py:4-72) loads the plugin by path, solves it in one
process and prints "Winning position", "Losing position", "Tie" or "Draw"
(:29-40).  As committed it prints "Draw" for every game: its result constants
are strings while plugins return src.utils ints (:6), and its TIE
branch tests LOSS twice (:34).  This drop-in prints the message the reference
intends for the root's canonical value, computed on the GPU by libgmsolve.so;
``--remoteness`` adds the launcher's "<V> in <R> moves" line.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import solver_launcher  # noqa: E402

MESSAGES = {0: "Winning position", 1: "Losing position", 2: "Tie", 3: "Draw"}


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("game_file")
    p.add_argument("--custom")
    p.add_argument("--init_pos")
    p.add_argument("--dims")
    p.add_argument("--heaps", type=int)
    p.add_argument("--remoteness", action="store_true")
    p.add_argument("--device", type=int, default=-1)
    args = p.parse_args(argv)
    args.engine = "auto"
    game, root = solver_launcher.prepare_game(args)
    from gamesmanmpi_amd import Solver
    s = Solver(game, root, device=args.device)
    s.solve()
    print(MESSAGES[s.value])
    if args.remoteness:
        print(s.root_line())
    s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
