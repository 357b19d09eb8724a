"""-sd tables in the reference's layout (gamesmanmpi_amd/persist.py; CacheDict,
reference src/cache_dict.py:19-42, owner hash src/game_state.py:23-31).  CPU only:
the tables written are the golden ones of the reference's own plugins."""
import hashlib
import os
import shelve

import numpy as np
import pytest

from conftest import golden
from gamesmanmpi_amd import games
from gamesmanmpi_amd.persist import owner_rank, read_reference_tables, write_reference_tables


@pytest.mark.parametrize("name,codec", [
    ("ttt", games.TTTStringCodec()), ("othello_4x4", games.OthelloCodec(4, 4)),
    ("four_to_one_six", games.FourToOneCodec()), ("toot_3x3", games.TootCodec(3, 3))])
@pytest.mark.parametrize("world", [1, 3])
def test_reference_layout_round_trip(tmp_path, name, codec, world):
    keys, recs = golden(name)
    counts = write_reference_tables(str(tmp_path), codec, keys, recs, world)
    assert sum(counts) == len(keys)
    back = read_reference_tables(str(tmp_path), world)
    assert len(back) == len(keys)
    for k, r in zip(keys.tolist()[::97], recs.tolist()[::97]):
        pos = codec.pos(k)
        assert back[pos] == (r >> 14, r & 0x3FFF)
    for r in range(world):   # CacheDict paths: <sd>/stats/<rank>/{resolved,remote}
        with shelve.open(os.path.join(str(tmp_path), "stats", str(r), "resolved"), flag="r") as db:
            for k in list(db.keys())[:50]:
                assert int(hashlib.md5(k.encode("utf-8")).hexdigest(), 16) % world == r


def test_reference_keys_are_the_plugin_positions(tmp_path):
    keys, recs = golden("ttt")
    write_reference_tables(str(tmp_path), games.TTTStringCodec(), keys, recs)
    back = read_reference_tables(str(tmp_path))
    assert back["_________"] == (2, 9)                  # TIE in 9 (reference mttt_test.py blank)
    assert owner_rank("_________", 2) == int(hashlib.md5(b"_________").hexdigest(), 16) % 2
    keys, recs = golden("four_to_one_four")
    write_reference_tables(str(tmp_path / "f2o"), games.FourToOneCodec(), keys, recs)
    assert read_reference_tables(str(tmp_path / "f2o"))["4"] == (0, 3)   # WIN in 3


def test_wide_keys_round_trip(tmp_path):
    """Keys past 64 bits (Othello 8x8: (n, 3) u64 word arrays from gm_export_key) are written
    as the plugin's position strings, like any other key."""
    from gamesmanmpi_amd import _lib, games
    from gamesmanmpi_amd.persist import read_reference_tables, write_reference_tables
    codec = games.OthelloCodec(8, 8)
    pos = [bytes.fromhex(h).decode("latin-1") for h in ("303800204018057a4646bfdebfe6fa800200",
                                                        "30380028503841784646bfd6afc6be000200")]
    keys = np.array([_lib.int_to_words(codec.key(p), 3) for p in pos], dtype=np.uint64)
    recs = np.array([(1 << 14) | 11, 13], dtype=np.uint16)
    counts = write_reference_tables(str(tmp_path), codec, keys, recs, 2)
    assert sum(counts) == 2
    back = read_reference_tables(str(tmp_path), 2)
    assert back == {pos[0]: (1, 11), pos[1]: (0, 13)}
