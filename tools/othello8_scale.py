#!/usr/bin/env python3
"""Othello 8x8 endgames on the device: solve the seed-5 playout's position
with E empty squares for each E given, on one GPU (and, with --ranks R, again with R virtual
ranks: the digests must agree), and print one JSON line per solve.

    python tools/othello8_scale.py 14 16 18 [--ranks 8] [--repeats 2]

The roots are the positions of the fixed random playout from the standard start that
tests/plugins/othello8_endgame.py documents (random.Random(5), a uniform legal move each ply;
10 empties = that plugin's default root), regenerated here with this repo's plugin."""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def playout_roots(seed=5):
    """Empty-square count -> the first position of the seed's playout with that many empties."""
    import test_games.othello_bit_new as o
    rng = random.Random(seed)
    p = o.initial_position()
    out = {}
    while o.primitive(p) == 4:
        ms = o.gen_moves(p)
        p = o.do_move(p, ms[rng.randrange(len(ms))])
        b = p.encode("latin-1")
        e = 64 - bin(int.from_bytes(b[0:8], "big") | int.from_bytes(b[8:16], "big")).count("1")
        out.setdefault(e, p)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("empties", type=int, nargs="+")
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--repeats", type=int, default=2)
    a = ap.parse_args()
    from gamesmanmpi_amd import Context, _lib, games
    codec = games.OthelloCodec(8, 8)
    roots = playout_roots()
    for e in a.empties:
        pos = roots[e]
        key = codec.key(pos)
        for ranks in sorted({1, a.ranks}):
            ctx = Context(_lib.GAME_OTHELLO, (8, 8), device=0)
            if ranks > 1:
                ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
            times = []
            for _ in range(a.repeats):
                t0 = time.perf_counter()
                n, rec = ctx.solve(key)
                times.append(time.perf_counter() - t0)
            st = ctx.stats()
            d, m = ctx.digest()
            print(json.dumps({"empties": e, "root_hex": pos.encode("latin-1").hex(), "ranks": ranks, "positions": n,
                              "root_record": rec, "solve_s": [round(t, 4) for t in times],
                              "positions_per_s": n / min(times), "forward_ms": st["forward_ms"],
                              "backward_ms": st["backward_ms"], "table_gb": st["table_bytes"] / 1e9,
                              "edges": st["n_edges"], "tiers": st["n_tiers"], "digest": "%#018x" % d,
                              "digest_positions": m}), flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
