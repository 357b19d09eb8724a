#!/usr/bin/env python3
"""Toot-and-Otto beyond 24 cells under the reference's rules.

    python tools/toot_stuck_positions.py [L H ...]

The reference gives each player 6 T and 6 O (the hand nibbles 0b0110,
test_games/toot_and_otto_bitstring.py:36-44), whatever the board.  On a board of more than
24 cells the 24 pieces can all be placed with TOOT and OTTO counts equal and the board not
full: the mover then has no move (gen_moves :87-99 needs a piece in hand) and the position
is not primitive (TIE only on a full board, :80-81) -- a non-primitive position without
children, where the reference's solver waits forever (new_process.py
_add_pending_state sets a zero counter that nothing resolves).  Random playouts under those
rules (a restatement, pure Python) find such positions on 5x5 and 7x4 within a few dozen
games; prints one per board.  Test infrastructure / documentation, not the product.
"""
import random
import sys


def words(b, L, H):
    sc = {"TOOT": 0, "OTTO": 0}
    for x in range(L):
        for y in range(H):
            for dx, dy in ((1, 0), (0, 1), (1, 1), (1, -1)):
                s = ""
                for i in range(4):
                    xx, yy = x + dx * i, y + dy * i
                    if not (0 <= xx < L and 0 <= yy < H):
                        break
                    s += b.get((xx, yy), "-")
                if s in sc:
                    sc[s] += 1
    return sc


def find_stuck(L, H, tries=2000, seed=1):
    """A reachable position (dict cell -> letter) with no move that is not primitive, or None."""
    rng = random.Random(seed)
    for t in range(tries):
        b, hands, h, p = {}, [[6, 6], [6, 6]], [0] * L, 0
        while True:
            sc = words(b, L, H)
            if sc["TOOT"] != sc["OTTO"]:
                break                                   # primitive: WIN / LOSS
            moves = [(x, c) for x in range(L) if h[x] < H for c, k in (("T", 0), ("O", 1)) if hands[p][k] > 0]
            if not moves:
                if len(b) < L * H:
                    return t + 1, b
                break                                   # full board, equal counts: TIE
            x, c = rng.choice(moves)
            b[(x, h[x])] = c
            h[x] += 1
            hands[p][0 if c == "T" else 1] -= 1
            p ^= 1
    return None


def main():
    args = [int(x) for x in sys.argv[1:]] or [5, 5, 7, 4]
    for L, H in zip(args[::2], args[1::2]):
        r = find_stuck(L, H)
        if r is None:
            print("%dx%d: no stuck position found" % (L, H))
            continue
        t, b = r
        print("%dx%d: after %d random games, %d pieces placed, both hands empty, board not full, "
              "TOOT == OTTO -- no move, not primitive:" % (L, H, t, len(b)))
        for y in reversed(range(H)):
            print("   " + " ".join(b.get((x, y), "-") for x in range(L)))


if __name__ == "__main__":
    main()
