#!/usr/bin/env python3
"""Generate the golden fixtures in ``tests/golden/`` from the REFERENCE's own plugins.

Run in the build container (``/root/reference`` present; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--live]

What it does:

1. imports the reference's ``src.utils`` and plugin modules from
   ``/root/reference/test_games`` (with an empty ``mpi4py`` stub for
   ``tic_tac_toe_np.py:2`` and ``bitstring_shim.BitArray`` standing in for the
   absent third-party ``bitstring`` package);
2. strong-solves them with the canonical fixed point of ``oracle/canonical.py``
    and writes, per config, the sorted ``(key u64, record u16)``
   table as ``<name>.npz`` (record = value << 14 | remoteness);
3. writes ``roots.json``: the root line for the 9 cases of the reference's
   ``game_tests/four_to_one_test.py`` and ``game_tests/mttt_test.py`` (custom roots
   loaded from ``game_tests/*_init_pos.py`` exactly as ``--custom/--init_pos``
   intends), next to the line those tests expect;
4. with ``--live``: also drives the reference's live engine
   (``src/new_process.Process`` + ``src/new_job.Job``) single-rank under an
   in-process fake MPI and records how its values / remoteness compare with the
   canonical table (``live.json``).

Keys:
  four_to_one: the pile as a signed int64 (stored two's complement in u64);
  ttt:         sum of c * 3**(x + 3y), c = 0 blank, 1 X / player 1, 2 O / player 2;
  toot:        the first 2A+16 bits of the position string (planes + hands), MSB-first;
  othello:     all 2A+16 bits of the position string, MSB-first;
  othello 8x8: the first 8 bytes of blake2b(position string bytes), big-endian (2A+16 = 144
               bits do not fit a u64; tests/plugins/othello8_endgame.py).

``--only othello8`` writes just the 8x8 endgame fixture (othello_8x8_endgame.npz) and its
entry in roots.json.
"""
import argparse
import importlib.util
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True


def _install_stubs():
    mpi4py = types.ModuleType("mpi4py")
    mpi4py.MPI = types.ModuleType("mpi4py.MPI")
    sys.modules["mpi4py"] = mpi4py
    sys.modules["mpi4py.MPI"] = mpi4py.MPI
    sys.path.insert(0, HERE)
    import bitstring_shim
    bs = types.ModuleType("bitstring")
    bs.BitArray = bitstring_shim.BitArray
    sys.modules["bitstring"] = bs
    cachetools = types.ModuleType("cachetools")

    class LRUCache(dict):
        def __init__(self, maxsize=None):
            super().__init__()
    cachetools.LRUCache = LRUCache
    sys.modules["cachetools"] = cachetools
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REPO, "oracle"))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def key_f2o(pos):
    return int(pos) & 0xFFFFFFFFFFFFFFFF


def key_ttt_str(pos):
    digit = {"_": 0, "X": 1, "O": 2}
    return sum(digit[ch] * 3 ** i for i, ch in enumerate(pos))


def key_ttt_np(state):
    return sum(int(state[x][y]) * 3 ** (x + 3 * y) for x in range(3) for y in range(3))


def key_bits(nkeep):
    def k(pos):
        raw = pos.encode("ISO-8859-1")
        v = int.from_bytes(raw, "big")
        return v >> (8 * len(raw) - nkeep)
    return k


def key_blake8(pos):
    import hashlib
    return int.from_bytes(hashlib.blake2b(pos.encode("ISO-8859-1"), digest_size=8).digest(), "big")


# tests/plugins/othello8_endgame.py's root: the reference's default 8x8 board after a fixed
# random playout from the start (seed 5), 10 empty squares left
OTHELLO8_ENDGAME_HEX = "303800204018057a4646bfdebfe6fa800200"


def othello8_endgame(canonical, ref_utils, roots):
    oth = _load("game_module", os.path.join(REF, "test_games/othello_bit_new.py"))   # 8x8 as shipped
    ref_utils.game_module = oth
    assert (oth.length, oth.height) == (8, 8)
    root = bytes.fromhex(OTHELLO8_ENDGAME_HEX).decode("latin-1")
    t0 = time.time()
    table, positions = canonical.solve(oth, root)
    save_table("othello_8x8_endgame", table, positions, key_blake8,
               {"game": "othello_bit_new", "dims": [8, 8], "root_hex": OTHELLO8_ENDGAME_HEX, "key": "blake2b-8"})
    v, r = table[canonical.default_key(root)]
    roots["othello_8x8_endgame"] = {"root_hex": OTHELLO8_ENDGAME_HEX, "canonical": canonical.root_line(v, r),
                                    "positions": len(table), "seconds": round(time.time() - t0, 1)}


def save_table(name, table, positions, keyfn, meta):
    keys = np.empty(len(table), dtype=np.uint64)
    recs = np.empty(len(table), dtype=np.uint16)
    for i, (k, (v, r)) in enumerate(table.items()):
        keys[i] = keyfn(positions[k])
        recs[i] = (v << 14) | r
    order = np.argsort(keys, kind="stable")
    keys, recs = keys[order], recs[order]
    if len(np.unique(keys)) != len(keys):
        raise SystemExit("%s: key collision" % name)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), keys=keys, records=recs,
                        meta=json.dumps(meta))
    vals = recs >> 14
    print("%-14s %9d positions  W %d  L %d  T %d" % (
        name, len(keys), (vals == 0).sum(), (vals == 1).sum(), (vals == 2).sum()))
    return keys, recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--live", action="store_true")
    ap.add_argument("--skip-big", action="store_true")
    ap.add_argument("--only", choices=("othello8",), default=None)
    args = ap.parse_args()
    _install_stubs()
    import canonical
    import src.utils as ref_utils

    roots = {}
    if args.only == "othello8":
        path = os.path.join(HERE, "roots.json")
        roots = json.load(open(path))
        othello8_endgame(canonical, ref_utils, roots)
        with open(path, "w") as f:
            json.dump(roots, f, indent=1, sort_keys=True)
        print(json.dumps(roots["othello_8x8_endgame"], indent=1))
        return

    def root_line(table, positions, root, keyfn=None):
        v, r = table[canonical.default_key(root)]
        return canonical.root_line(v, r)

    # ---- Four-To-One (config 1) and the four golden roots --------------------
    f2o = _load("game_module", os.path.join(REF, "test_games/four_to_one.py"))
    ref_utils.game_module = f2o
    f2o_roots = _load("custom_f2o", os.path.join(REF, "game_tests/four_to_one_init_pos.py"))
    expect_f2o = {"four": (None, "WIN in 3 moves"), "six": ("six", "LOSS in 4 moves"),
                  "one": ("one", "WIN in 1 moves"), "zero": ("zero", "LOSS in 0 moves")}
    for case, (attr, expected) in expect_f2o.items():
        root = f2o.initial_position() if attr is None else getattr(f2o_roots, attr)()
        table, positions = canonical.solve(f2o, root)
        save_table("four_to_one_%s" % case, table, positions, key_f2o,
                   {"game": "four_to_one", "root": root})
        roots["four_to_one/%s" % case] = {
            "root": root, "canonical": root_line(table, positions, root),
            "reference_test_expects": expected,
            "test": "game_tests/four_to_one_test.py::test_%s" % case}

    # ---- mttt (config 2 twin) + the five golden roots ------------------------
    mttt = _load("game_module", os.path.join(REF, "test_games/mttt.py"))
    ref_utils.game_module = mttt
    mttt_roots = _load("custom_mttt", os.path.join(REF, "game_tests/mttt_test_init_pos.py"))
    table, positions = canonical.solve(mttt)
    ttt_keys, ttt_recs = save_table("ttt", table, positions, key_ttt_str,
                                    {"game": "mttt", "root": mttt.initial_position()})
    expect_mttt = {"blank": (None, "TIE in 9 moves"), "tie_in_one": ("tie_in_one", "TIE in 1 moves"),
                   "win_in_one": ("win_in_one", "WIN in 1 moves"),
                   "side_columns": ("side_columns", "TIE in 3 moves"),
                   "one_row": ("one_row", "TIE in 3 moves")}
    for case, (attr, expected) in expect_mttt.items():
        root = mttt.initial_position() if attr is None else getattr(mttt_roots, attr)()
        t2, p2 = canonical.solve(mttt, root)
        roots["mttt/%s" % case] = {
            "root": root, "root_key": key_ttt_str(root), "positions": len(t2),
            "canonical": root_line(t2, p2, root), "reference_test_expects": expected,
            "test": "game_tests/mttt_test.py::test_%s" % case}
        if case != "blank":
            save_table("mttt_%s" % case, t2, p2, key_ttt_str, {"game": "mttt", "root": root})

    # ---- tic_tac_toe_np (config 2) -----------------------------------------
    ttt_np = _load("game_module", os.path.join(REF, "test_games/tic_tac_toe_np.py"))
    ref_utils.game_module = ttt_np
    table, positions = canonical.solve(ttt_np)
    k2, r2 = save_table("ttt_np", table, positions, key_ttt_np, {"game": "tic_tac_toe_np"})
    if not (np.array_equal(k2, ttt_keys) and np.array_equal(r2, ttt_recs)):
        raise SystemExit("mttt and tic_tac_toe_np tables differ")

    # ---- Othello 4x4 (config 4) ---------------------------------------------
    oth = _load("game_module", os.path.join(REF, "test_games/othello_bit_new.py"))
    ref_utils.game_module = oth
    oth.length, oth.height = 4, 4
    oth.area = 16
    t0 = time.time()
    table, positions = canonical.solve(oth)
    root = oth.initial_position()
    save_table("othello_4x4", table, positions, key_bits(48),
               {"game": "othello_bit_new", "dims": [4, 4], "root_hex": root.encode("latin-1").hex()})
    roots["othello_4x4"] = {"root_hex": root.encode("latin-1").hex(),
                            "canonical": root_line(table, positions, root),
                            "positions": len(table), "seconds": round(time.time() - t0, 1)}

    # ---- Toot-and-Otto (config 3, small boards) ------------------------------
    toot = _load("game_module", os.path.join(REF, "test_games/toot_and_otto_bitstring.py"))
    ref_utils.game_module = toot
    toot_dims = [(3, 3), (4, 3)] if not args.skip_big else [(3, 3)]
    for (L, H) in toot_dims:
        toot.length, toot.height, toot.area = L, H, L * H
        t0 = time.time()
        table, positions = canonical.solve(toot)
        root = toot.initial_position()
        name = "toot_%dx%d" % (L, H)
        save_table(name, table, positions, key_bits(2 * L * H + 16),
                   {"game": "toot_and_otto_bitstring", "dims": [L, H],
                    "root_hex": root.encode("latin-1").hex()})
        roots[name] = {"root_hex": root.encode("latin-1").hex(),
                       "canonical": root_line(table, positions, root),
                       "positions": len(table), "seconds": round(time.time() - t0, 1)}

    othello8_endgame(canonical, ref_utils, roots)

    with open(os.path.join(HERE, "roots.json"), "w") as f:
        json.dump(roots, f, indent=1, sort_keys=True)
    print(json.dumps(roots, indent=1, sort_keys=True))

    if args.live:
        import live_reference
        out = live_reference.run_all(_load, canonical, ref_utils)
        with open(os.path.join(HERE, "live.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
