"""CPU checks of the C-ABI library: it loads, exports what include/gmsolve.h declares,
and its host-side descriptor twins agree with the oracle.  No device work here, except the
gpu-marked gm_query test (the documented answer of each engine)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO, golden, load_plugin
from gamesmanmpi_amd import _lib, games

F2O, TTT, TOOT, OTH, SUB = 1, 2, 3, 4, 5


def header_symbols():
    text = open(os.path.join(REPO, "include", "gmsolve.h")).read()
    return set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gm_\w+)\s*\(", text, re.M))


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    declared = header_symbols()
    assert declared == set(_lib.SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gm_\w+)", out))
    assert declared <= exported
    for name in declared:
        assert getattr(lib, name) is not None
    assert lib.gm_version() == 2


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH],
                         capture_output=True, text=True, cwd="/tmp")
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_no_gpu_means_loud_failure():
    if _lib.lib().gm_device_count() > 0:
        pytest.skip("a GPU is visible")
    from gamesmanmpi_amd import Context, GMError
    ctx = Context(TTT, ())
    with pytest.raises(GMError, match="no HIP device"):
        ctx.solve(0)


def test_open_rejects_bad_games():
    from gamesmanmpi_amd import Context, GMError
    for game, params in [(99, ()), (TOOT, (9, 4)), (OTH, (4, 3)), (SUB, (9,)), (OTH, (6, 6))]:
        with pytest.raises(GMError):
            Context(game, params)


@pytest.mark.parametrize("game,params", [(F2O, ()), (TTT, ()), (TOOT, (6, 4)), (TOOT, (4, 3)),
                                         (OTH, (4, 4)), (SUB, (8,)), (SUB, (3,))])
def test_initial_keys_match_oracle(oracle, game, params):
    from gamesmanmpi_amd import Context
    assert Context(game, params).initial() == oracle.initial(game, params)


@pytest.mark.parametrize("name,codec", [
    ("ttt", games.TTTStringCodec()), ("othello_4x4", games.OthelloCodec(4, 4)),
    ("toot_3x3", games.TootCodec(3, 3)), ("toot_4x3", games.TootCodec(4, 3)),
    ("four_to_one_six", games.FourToOneCodec())])
def test_descriptor_host_twin_matches_oracle_on_golden_positions(oracle, name, codec):
    hd = games.HostDescriptor(codec)
    keys, _ = golden(name)
    step = max(1, len(keys) // 20000)
    for k in keys[::step].tolist():
        p1, c1, t1 = hd.expand(k)
        assert (p1, sorted(c1), t1) == oracle.expand(codec.game_id, codec.params, k), hex(k)


def test_toot_6x4_descriptor_random_playouts(oracle):
    codec = games.TootCodec(6, 4)
    hd = games.HostDescriptor(codec)
    rng = np.random.default_rng(3)
    for _ in range(300):
        k = hd.initial()
        while True:
            p, kids, t = hd.expand(k)
            assert (p, sorted(kids), t) == oracle.expand(TOOT, (6, 4), k)
            if not kids:
                break
            k = kids[rng.integers(len(kids))]


def test_expand_rejects_invalid_keys():
    hd = games.HostDescriptor(games.OthelloCodec(4, 4))
    with pytest.raises(_lib.GMError):
        hd.expand(0)           # turn byte 0 is not a position


@pytest.mark.parametrize("rel,attrs,name,params", [
    ("test_games/four_to_one.py", {}, "four_to_one", ()),
    ("test_games/mttt.py", {}, "mttt", ()),
    ("test_games/tic_tac_toe_np.py", {}, "tic_tac_toe_np", ()),
    ("test_games/toot_and_otto_bitstring.py", {}, "toot_and_otto", (6, 4)),
    ("test_games/toot_and_otto_bitstring.py", {"length": 4, "height": 3}, "toot_and_otto", (4, 3)),
    ("test_games/othello_bit_new.py", {"length": 4, "height": 4}, "othello", (4, 4)),
    ("test_games/subtraction.py", {}, "subtraction", (8,)),
])
def test_identify_plugins(rel, attrs, name, params):
    mod = load_plugin(rel, **attrs)
    c = games.identify(mod)
    assert c is not None and c.name == name and tuple(c.params) == params
    root = mod.initial_position()
    assert c.key(c.pos(c.key(root))) == c.key(root)


def test_identify_rejects_a_modified_game():
    mod = load_plugin("test_games/mttt.py")
    orig = mod.primitive

    def misere(pos):      # a different game: full board is a LOSS instead of a TIE
        v = orig(pos)
        return 1 if v == 2 else v
    mod.primitive = misere
    assert games.identify(mod) is None


def test_identify_needs_certainty_not_a_sample():
    """A plugin equal to mttt on every board of up to 6 pieces (all that the sampled
    check sees first) must not bind to the TTT descriptor (exhaustive check,
    games.identify); the sampled check alone would accept it."""
    mod = load_plugin("tests/plugins/mttt_late_rule.py")
    assert games.verify(mod, games.TTTStringCodec(), mod.initial_position(), samples=0)
    assert games.identify(mod) is None


def test_identify_binds_an_unknown_but_equal_plugin_exhaustively():
    """mttt's rules rewritten (different code, same game): no known fingerprint, but
    every reachable position agrees, so it binds -- and not when the exhaustive
    check is capped below the game's 5,478 positions."""
    mod = load_plugin("tests/plugins/mttt_late_rule.py")
    orig = mod.primitive
    mod.primitive = lambda pos: 1 if orig(pos) == 0 else orig(pos)   # WIN -> LOSS: exactly mttt
    c = games.identify(mod)
    assert c is not None and c.name == "mttt"
    assert games.identify(mod, exhaustive_max=1000) is None


def test_fingerprints_cover_this_repos_plugins():
    """plugin_fingerprints.json is current (python -m gamesmanmpi_amd.fingerprint --write)."""
    from gamesmanmpi_amd import fingerprint as fp
    known = fp.known()
    for rel, codec in fp.SOURCES:
        got = known.get(fp.fingerprint(load_plugin(rel)))
        assert got is not None and got["codec"] == codec, rel
    # dimensions are parameters, not code: a patched board keeps its fingerprint
    assert fp.fingerprint(load_plugin("test_games/othello_bit_new.py", length=4, height=4)) == \
        fp.fingerprint(load_plugin("test_games/othello_bit_new.py"))


def test_launcher_custom_root_keeps_the_fingerprint_binding():
    """`solver_launcher.py GAME --custom FILE --init_pos NAME` replaces the module's
    initial_position (as the reference's launcher does, solver_launcher.py:106-111); the rules
    are unchanged, so the 8x8 plugin still binds the 128-bit-key descriptor by its fingerprint
    and not through the exhaustive replay, which is capped at 10^6 positions (a 16-empty root
    has 1.48 G below it)."""
    import solver_launcher
    from gamesmanmpi_amd import fingerprint as fp
    args = solver_launcher.build_parser().parse_args(
        [os.path.join(REPO, "test_games/othello_bit_new.py"), "--custom",
         os.path.join(REPO, "tools/othello8_roots.py"), "--init_pos", "endgame_16"])
    game, root = solver_launcher.prepare_game(args)
    assert game.initial_position.__name__ == "endgame_16" and len(root) == 18
    assert fp.known().get(fp.fingerprint(game), {}).get("codec") == "othello"
    c = games.identify(game, root, exhaustive_max=0)
    assert c is not None and c.name == "othello" and c.params == (8, 8)


def test_othello_8x8_binds_the_wide_descriptor():
    """the reference plugin at its default 8x8 board (othello_bit_new.py:8,
    144-bit positions) binds to the 128-bit-key descriptor (games.hpp DescOthello8): 3 key words,
    the initial key is the plugin's initial position string as an integer, and the host twin
    agrees with the plugin (primitive value and child set) on EVERY one of the 56,552 positions
    below the seed-5 endgame root (tests/plugins/othello8_endgame.py)."""
    mod = load_plugin("test_games/othello_bit_new.py")     # reference default 8x8
    c = games.identify(mod)
    assert c is not None and c.name == "othello" and c.params == (8, 8)
    hd = games.HostDescriptor(c)
    assert hd.words == 3 and hd.initial() == c.key(mod.initial_position())
    hd.close()
    end = load_plugin("tests/plugins/othello8_endgame.py")
    ce = games.identify(end)
    assert ce is not None and ce.params == (8, 8)
    assert games.verify_exhaustive(end, ce, end.initial_position(), 100_000)


def test_othello_8x8_bitboard_moves_vs_plugin_on_random_games():
    """The bitboard move generator of the 8x8 descriptor (games.hpp DescOthello8::legal /
    flips_at, the code the device kernels run) against the plugin over WHOLE games: seeded
    random playouts from the 8x8 start, every position's primitive value and child set (the
    endgame test above only sees near-full boards)."""
    import random
    mod = load_plugin("test_games/othello_bit_new.py")
    c = games.identify(mod)
    hd = games.HostDescriptor(c)
    rng = random.Random(11)
    n = passes = 0
    for _ in range(150):
        p = mod.initial_position()
        while True:
            prim, kids, _ = hd.expand(c.key(p))
            assert prim == mod.primitive(p)
            if prim != 4:
                break
            ch = [mod.do_move(p, m) for m in mod.gen_moves(p)]
            assert sorted(kids) == sorted(c.key(x) for x in ch)
            n += 1
            passes += len(ch) == 1 and mod.gen_moves(p) == [None]
            p = ch[rng.randrange(len(ch))]
    hd.close()
    assert n > 8000 and passes > 0


def test_othello_8x8_key_words_round_trip():
    """gm_expand_host_key rejects a key that is no 8x8 position (a centre square empty, planes
    overlapping, turn 3), and the one-word calls refuse a 3-word context."""
    from gamesmanmpi_amd import Context, GMError
    ctx = Context(OTH, (8, 8))
    assert ctx.words == 3
    k = ctx.initial()
    hd = games.HostDescriptor(games.OthelloCodec(8, 8))
    prim, kids, tier = hd.expand(k)
    assert prim == 4 and len(kids) == 4 and tier == 3 * 4
    for bad in (k & ~(1 << (80 + 63 - 27)) & ~(1 << (16 + 63 - 27)),   # centre square (3, 3) emptied
                k | (1 << (16 + 63 - 27)),                                  # (3, 3) white and black
                (k & ~(0xFF << 8)) | (3 << 8)):                             # turn byte 3
        with pytest.raises(GMError, match="valid"):
            hd.expand(bad)
    with pytest.raises(GMError, match="3 words"):
        _lib.check(ctx.L.gm_pack_initial(ctx.h, ctypes.byref(ctypes.c_uint64())))
    hd.close()
    ctx.close()


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present (GPU box)")
@pytest.mark.parametrize("rel,name", [("test_games/mttt.py", "mttt"), ("test_games/four_to_one.py", "four_to_one")])
def test_reference_plugin_files_route_to_descriptors(rel, name):
    """Unmodified reference plugins import our src.utils and match a descriptor."""
    mod = load_plugin(os.path.join(REF, rel))
    c = games.identify(mod)
    assert c is not None and c.name == name


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["box", "box_virtual_ranks", "block", "sparse"])
def test_query_semantics_per_engine(oracle, engine):
    """gm_query as include/gmsolve.h documents it, per engine, on one GPU
    (a rank of a multi-process split answers only its own boxes' keys:
    tests/test_gpu_multiproc.py::test_box_rccl_custom_root_vs_oracle).  Every key of the
    solved set answers the oracle's record; a key outside it answers 0xFFFF."""
    from gamesmanmpi_amd import Context
    if engine == "sparse":
        game, params, root = TOOT, (4, 3), None
    else:
        game, params, root = SUB, (8,), 0x33557777
    ctx = Context(game, params, device=0)
    if engine == "box_virtual_ranks":
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, 4)
    elif engine == "block":
        ctx.set_option(_lib.OPT_SUB_INTERLEAVE, 10)
    if root is None:
        root = ctx.initial()
    ctx.solve(root)
    ok, orec = oracle.solve(game, params, root=root)
    step = max(1, len(ok) // 5000)
    assert np.array_equal(ctx.query(ok[::step]), orec[::step])
    if engine == "sparse":
        outside = np.setdiff1d(np.arange(int(ok.max()) + 1, int(ok.max()) + 64, dtype=np.uint64), ok)[:8]
    else:
        outside = np.array([0x33557778, 0x43557777, 0xFFFFFFFF, 1 << 32], dtype=np.uint64)
    assert ctx.query(outside).tolist() == [_lib.REC_UNSOLVED] * len(outside)
    ctx.close()


def test_header_documents_query_per_engine():
    """The header's gm_query comment names the rule for each engine."""
    text = open(os.path.join(REPO, "include", "gmsolve.h")).read()
    doc = text[:text.index("int gm_query(")].rsplit("/*", 1)[1]
    for phrase in ("0xFFFF", "multi-process", "box engine", "sparse", "virtual ranks"):
        assert phrase in doc, phrase


def test_abi_layout_pinned(tmp_path):
    """GM_ABI_VERSION 2 pins the struct and the signatures a ctypes caller relies
    on.  gcc compiles the header and prints sizeof / offsetof of gm_stats_t; they equal the
    ctypes mirror's.  gm_box_plan carries its opts and axis parameters, gm_rank_stats its
    recv_bytes array."""
    import ctypes
    fields = [n for n, _ in _lib.Stats._fields_]
    src = tmp_path / "pin.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gmsolve.h"\nint main(void){\n'
                   '  printf("%zu\\n", sizeof(gm_stats_t));\n'
                   + "".join('  printf("%%zu\\n", offsetof(gm_stats_t, %s));\n' % f for f in fields)
                   + '  printf("%d\\n", GM_ABI_VERSION);\n  return 0;\n}\n')
    exe = tmp_path / "pin"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_lib.Stats)
    assert vals[1:-1] == [getattr(_lib.Stats, f).offset for f in fields]
    assert vals[-1] == _lib.ABI_VERSION == _lib.lib().gm_version()
    text = open(os.path.join(REPO, "include", "gmsolve.h")).read()
    assert re.search(r"int gm_box_plan\(uint64_t root_key, int world, int rank, const int32_t \*opts, int what, "
                     r"int axis, uint32_t \*out,\s+uint64_t cap, uint64_t \*n\);", text)
    assert re.search(r"int gm_rank_stats\(gm_ctx \*ctx, double \*kernel_ms, uint64_t \*boxes, uint64_t \*recv_bytes,",
                     text)
    assert len(_lib.lib().gm_box_plan.argtypes) == 9
