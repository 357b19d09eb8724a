"""Digest fixtures for boards too large to commit as tables.

    python tests/golden/make_oracle_digests.py

Runs the C oracle (oracle/gm_oracle.c, itself pinned to the reference plugins'
golden tables by tests/test_oracle_golden.py) on Toot-and-Otto 5x4 and 4x4 and
writes, per board, the position count, the per-ply counts and the
order-independent digest of the full (key, record) table (the gm_digest formula,
include/gmsolve.h) into tests/golden/oracle_digests.json.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import Oracle, digest  # noqa: E402

TOOT = 3


def main():
    o = Oracle()
    out = {}
    for L, H in ((4, 4), (5, 4)):
        t = time.time()
        keys, recs = o.solve(TOOT, (L, H))
        plies = np.zeros(L * H + 1, dtype=np.int64)
        planes = (keys >> np.uint64(16)) & np.uint64((1 << (2 * L * H)) - 1)
        pieces = np.array([bin(int(p)).count("1") for p in planes]) if len(keys) < 5_000_000 else None
        if pieces is None:   # popcount in chunks for the big board
            pieces = np.zeros(len(keys), dtype=np.int64)
            x = planes.copy()
            while x.any():
                pieces += (x & np.uint64(1)).astype(np.int64)
                x >>= np.uint64(1)
        np.add.at(plies, pieces, 1)
        root = int(recs[np.searchsorted(keys, np.uint64(o.initial(TOOT, (L, H))))])
        out["toot_%dx%d" % (L, H)] = {"positions": int(len(keys)), "per_ply": plies.tolist(),
                                     "digest": digest(keys, recs), "root_record": root}
        print("toot %dx%d: %d positions, %.1f s" % (L, H, len(keys), time.time() - t), flush=True)
    with open(os.path.join(HERE, "oracle_digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
