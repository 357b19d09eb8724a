"""Digest fixtures for tables too large to commit.

    python tests/golden/make_oracle_digests.py [board ...]

Runs the C oracle (oracle/gm_oracle.c, itself pinned to the reference plugins'
golden tables by tests/test_oracle_golden.py) and writes, per case, the position
count, the per-tier counts, the root record and the order-independent digest of
the full (key, record) table (the gm_digest formula, include/gmsolve.h) into
tests/golden/oracle_digests.json:

  toot_4x4, toot_5x4, toot_6x4   Toot-and-Otto (config 3 is 6x4: 1,187,212,827
                                 positions) by oracle_solve_layered, the sorted-layer
                                 OpenMP solver (6x4 needs ~25 GB of host memory);
                                 4x4 / 5x4 were first produced by the hash-map
                                 oracle_solve and both solvers agree on them;
  othello_4x4                    config 4 (54,089 positions; also a golden table);
  subtract_8                     the 2^32-position synthetic game (config 5) by
                                 oracle_subtract_dense_mt + oracle_dense_digest.

Existing entries are kept unless named on the command line.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import Oracle  # noqa: E402

TOOT, SUB = 3, 5
OUT = os.path.join(HERE, "oracle_digests.json")


def layered(o, game, params):
    n, dg, root, tiers = o.solve_layered(game, params)
    return {"positions": n, "per_tier": tiers, "digest": dg, "root_record": root}


def toot(o, L, H):
    n, dg, root, tiers = o.solve_layered(TOOT, (L, H))
    return {"positions": n, "per_ply": tiers, "digest": dg, "root_record": root}


def subtract(o, heaps):
    recs = o.subtract_dense_mt(heaps)
    dg = o.dense_digest(recs)
    root = int(recs[(1 << (4 * heaps)) - 1])
    del recs
    return {"positions": 1 << (4 * heaps), "digest": dg, "root_record": root}


CASES = {
    "othello_4x4": lambda o: layered(o, 4, (4, 4)),
    "toot_4x4": lambda o: toot(o, 4, 4),
    "toot_5x4": lambda o: toot(o, 5, 4),
    "toot_6x4": lambda o: toot(o, 6, 4),
    "subtract_8": lambda o: subtract(o, 8),
}


def main():
    names = sys.argv[1:] or list(CASES)
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    o = Oracle()
    for name in names:
        t = time.time()
        out[name] = CASES[name](o)
        print("%s: %d positions, root %#x, %.1f s" % (name, out[name]["positions"], out[name]["root_record"],
                                                     time.time() - t), flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
