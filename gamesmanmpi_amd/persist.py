"""Solved tables in the reference's on-disk layout.

The reference keeps two shelve databases per rank (``CacheDict``,
src/cache_dict.py:19-42, opened at src/new_process.py:76-77):

    <statsdir>/stats/<rank>/resolved     str(pos) -> value code (src/utils.py:4)
    <statsdir>/stats/<rank>/remote       str(pos) -> remoteness

where a position lives on rank ``md5(str(pos)) % world_size``
(GameState.get_hash, src/game_state.py:23-31) and int keys are stringified
(src/cache_dict.py:62-66).  ``write_reference_tables`` writes a solved table
(``gm_export``: sorted u64 keys + u16 records; ``gm_export_key``'s (n, words) arrays for
keys past 64 bits) in that layout, so tooling that
reads the reference's ``-sd`` directory reads ours; ``read_reference_tables``
reads it back (tests, and resuming from a reference run's tables).
"""
import hashlib
import os
import shelve

import numpy as np

from . import _lib


def owner_rank(pos, world_size):
    """The reference's owner hash (src/game_state.py:23-31)."""
    return int(hashlib.md5(str(pos).encode("utf-8")).hexdigest(), 16) % world_size


def shelf_key(pos):
    """CacheDict's key for a position: ints and numpy boards as str (src/cache_dict.py:62-66)."""
    return pos if isinstance(pos, str) else str(pos)


def _path(statsdir, rank, name):
    d = os.path.join(statsdir or "", "stats", str(rank))
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, name)


def write_reference_tables(statsdir, codec, keys, records, world_size=1):
    """Write (keys, records) as the reference's per-rank resolved/remote shelves.

    ``codec`` maps keys back to plugin positions (gamesmanmpi_amd.games).  Returns the
    number of positions written per rank.
    """
    keys = np.asarray(keys, dtype=np.uint64)
    records = np.asarray(records, dtype=np.uint16)
    # keys past 64 bits (Othello 8x8) come as (n, words) u64 arrays: one Python int each
    key_list = [_lib.words_to_int(w) for w in keys.tolist()] if keys.ndim == 2 else keys.tolist()
    shelves = []
    for r in range(world_size):
        shelves.append((shelve.open(_path(statsdir, r, "resolved")), shelve.open(_path(statsdir, r, "remote"))))
    counts = [0] * world_size
    try:
        for k, rec in zip(key_list, records.tolist()):
            if rec == _lib.REC_UNSOLVED:
                continue
            for pos in (codec.members(k) if hasattr(codec, "members") else (codec.pos(k),)):
                r = owner_rank(pos, world_size)   # a symmetric graph key stands for its whole orbit
                sk = shelf_key(pos)
                shelves[r][0][sk] = rec >> 14
                shelves[r][1][sk] = rec & 0x3FFF
                counts[r] += 1
    finally:
        for a, b in shelves:
            a.close()
            b.close()
    return counts


def read_reference_tables(statsdir, world_size=1):
    """{str(pos): (value, remoteness)} from a reference-layout stats directory."""
    out = {}
    for r in range(world_size):
        with shelve.open(_path(statsdir, r, "resolved"), flag="r") as res, \
                shelve.open(_path(statsdir, r, "remote"), flag="r") as rem:
            for k in res.keys():
                out[k] = (res[k], rem[k])
    return out
