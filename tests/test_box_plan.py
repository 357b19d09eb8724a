"""The sharded box solve's plan, checked on the CPU (no GPU needed).

At N > 1 the 8-heap subtraction game runs on the box engine (csrc/dense_box.hip), each
rank computing one member of every orbit of a group H of heap permutations and reading a
child box it does not compute from its image under some h in H, which it computed in the
same box-tier.  The plan comes from the product through gm_box_plan (the
host code gm_solve runs).  Checked here: the owned lists partition the root's region,
every child read resolves to a box of the rank's own earlier box-tier in the form the
kernel implements, the ranks' loads are equal per box-tier, and -- position by position,
in numpy -- a rank that solves only its boxes and reads through the plan's permutations
reproduces the C oracle's table.  Reference: the owner hash these plans replace,
src/game_state.py:23-31, and the child/result exchange they make unnecessary,
src/new_process.py:145-187.
"""
import numpy as np
import pytest

from gamesmanmpi_amd import _lib

FULL = 0xFFFFFFFF


def coords(b):
    b = np.asarray(b, dtype=np.int64)
    return [(b >> (2 * i)) & 3 for i in range(4)] + [(b >> (8 + 3 * j)) & 7 for j in range(4)]


def unit(d):
    return 1 << (2 * d) if d < 4 else 1 << (8 + 3 * (d - 4))


def bsym_box(code, b):
    """Restatement of csrc/dense_box.hip bsym_box: r^k rotates heaps 0-3 (heap i -> i + k),
    t swaps heaps 4/5 and 6/7."""
    b = np.asarray(b, dtype=np.int64)
    code = np.asarray(code, dtype=np.int64)
    k = code & 3
    f = b & 0xFF
    f = ((f | (f << 8)) >> (8 - 2 * k)) & 0xFF
    b = (b & ~0xFF) | f
    x = ((b >> 3) ^ b) & 0x1C700
    return np.where(code & 4, b ^ x ^ (x << 3), b)


def bsym_key(code, key):
    """Restatement of bsym_key on keys (heap i at bits 4 i)."""
    key = np.asarray(key, dtype=np.int64)
    code = np.asarray(code, dtype=np.int64)
    k = code & 3
    lo = key & 0xFFFF
    key = (key & 0xFFFF0000) | (((lo | (lo << 16)) >> (16 - 4 * k)) & 0xFFFF)
    x = ((key >> 4) ^ key) & 0x0F0F0000
    return np.where(code & 4, key ^ x ^ (x << 4), key)


def box_of_key(key):
    key = np.asarray(key, dtype=np.int64)
    b = np.zeros_like(key)
    for i in range(4):
        b |= ((key >> (4 * i + 2)) & 3) << (2 * i)
    for j in range(4):
        b |= ((key >> (16 + 4 * j + 1)) & 7) << (8 + 3 * j)
    return b


def region(root):
    lim = coords(box_of_key(root))
    b = np.arange(1 << 20, dtype=np.int64)
    c = coords(b)
    ok = np.ones(len(b), bool)
    for i in range(8):
        ok &= c[i] <= lim[i]
    return b[ok]


def plan(world, rank, root=FULL):
    P = {}
    for name, what in (("shape", _lib.BOXPLAN_SHAPE), ("boxes", _lib.BOXPLAN_BOXES), ("fills", _lib.BOXPLAN_FILLS),
                       ("off", _lib.BOXPLAN_TIER_OFF), ("own", _lib.BOXPLAN_OWN), ("map", _lib.BOXPLAN_MAP)):
        P[name] = _lib.box_plan(world, rank, what, root).astype(np.int64)
    return P


INVARIANT_ROOTS = [FULL, 0x33337777, 0x5577BBBB, 0x2211FFFF]


@pytest.mark.parametrize("root", [FULL, 0x33337777, 0x23457777, 0x0F0FFFFF])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_owned_lists_partition_the_region(world, root):
    reg = region(root)
    seen = np.zeros(1 << 20, np.int64)
    for r in range(world):
        p = plan(world, r, root)
        seen[p["own"]] += 1
        assert np.all(np.diff(p["own"]) > 0)
        # a rank owns only boxes it computes
        assert np.isin(p["own"], p["boxes"]).all()
    assert (seen[reg] == 1).all() and seen.sum() == len(reg)


@pytest.mark.parametrize("root", [FULL, 0x33337777, 0x23457777, 0x0F0FFFFF, 0x5577BBBB])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_every_child_read_is_an_own_box_of_the_tier_below(world, root):
    """The kernel's contract (bx_issue): a child of a computed box along heap d is read from
    bsym_box(code, C) with code the fill's 3 bits at 3 d; that box must be one this rank
    computes in the box-tier before (an earlier launch), and the code must be a rotation
    for an A child (an address change) and t for a B child (a byte shuffle)."""
    for r in range(world):
        p = plan(world, r, root)
        boxes, fills, off = p["boxes"], p["fills"], p["off"]
        tier_of = np.full(1 << 20, -1, np.int64)
        for t in range(len(off) - 1):
            tier_of[boxes[off[t]:off[t + 1]]] = t
        c = coords(boxes)
        tier = sum(c)
        assert (tier_of[boxes] == tier).all()   # box-tier t holds the boxes of coordinate sum t
        for d in range(8):
            has = c[d] >= 1
            code = (fills >> (3 * d)) & 7
            assert (code[~has] == 0).all()
            if d < 4:
                assert (code & 4 == 0).all()
            else:
                assert (code & 3 == 0).all()
            src = bsym_box(code[has], boxes[has] - unit(d))
            assert (tier_of[src] == tier[has] - 1).all(), (r, d)


@pytest.mark.parametrize("world,boxes,ties", [(1, 1 << 20, 0), (2, 532480, 16384), (4, 282880, 40960),
                                              (8, 145600, 24640)])
def test_equal_loads_per_box_tier_and_redundancy(world, boxes, ties):
    """Every rank computes the same number of boxes in every box-tier (each rank's set is a
    heap permutation of the others'); only tie boxes (fixed by some h != id) are computed by
    more than one rank: 1.6 %, 7.9 %, 11.1 % more than an even share at 2, 4, 8 ranks."""
    per = None
    for r in range(world):
        p = plan(world, r)
        nsym, g, nb, nown, nties, ntiers = p["shape"].tolist()
        assert (nsym, nb, nties, ntiers) == (world, boxes, ties, 41)
        counts = np.diff(p["off"])
        per = counts if per is None else per
        assert np.array_equal(counts, per)
    assert per.sum() == boxes


@pytest.mark.parametrize("world", [2, 4, 8])
def test_query_map_sends_every_box_to_a_computed_image(world):
    reg = region(FULL)
    for r in range(world):
        p = plan(world, r)
        mine = np.zeros(1 << 20, bool)
        mine[p["boxes"]] = True
        m = p["map"]
        assert (m[reg] != 0xFF).all()
        assert mine[bsym_box(m[reg], reg)].all()
        out = np.ones(1 << 20, bool)
        out[reg] = False
        assert (m[out] == 0xFF).all()


def test_uninvariant_root_uses_the_stabiliser():
    """A root whose region no rotation maps onto itself keeps only the permutations that
    do (here t alone): 8 ranks then form 2 distinct sets, each computed by 4 ranks."""
    root = 0x777737BF   # A heaps 15, 11, 7, 3 (box coordinates 3, 2, 1, 0); B heaps all 7
    for r in range(8):
        nsym, g, nb, nown, nties, ntiers = plan(8, r, root)["shape"].tolist()
        assert nsym == 2 and g == (4 if r % 2 else 0)
        assert (nown > 0) == (r < 2)


def _emulate_rank(root, world, rank, p):
    """Solve rank `rank`'s boxes position by position (heap-sum order) in numpy, reading a
    child outside its boxes through the plan's permutation for that heap; returns the keys
    of its boxes and their 1-byte codes (csrc/gm_common.hpp)."""
    boxes = p["boxes"]
    fill_of = np.zeros(1 << 20, np.int64)
    fill_of[boxes] = p["fills"]
    mine = np.zeros(1 << 20, bool)
    mine[boxes] = True
    lim = [(root >> (4 * i)) & 15 for i in range(8)]
    stride = np.cumprod([1] + [lim[i] + 1 for i in range(7)])

    def cidx(k):   # compact index of a key of the root's region
        return sum(((k >> (4 * i)) & 15) * int(stride[i]) for i in range(8))

    # every key of the rank's boxes
    off = np.arange(4096, dtype=np.int64)
    c = coords(boxes)
    keys = np.zeros((len(boxes), 4096), np.int64)
    for i in range(4):
        keys |= ((c[i][:, None] << 2) | ((off[None, :] >> (4 + 2 * i)) & 3)) << (4 * i)
    for j in range(4):
        keys |= ((c[4 + j][:, None] << 1) | ((off[None, :] >> j) & 1)) << (16 + 4 * j)
    keys = np.sort(keys.ravel())
    h = [(keys >> (4 * i)) & 15 for i in range(8)]
    assert all((h[i] <= lim[i]).all() for i in range(8))
    level = sum(h)
    val = np.zeros(int(stride[-1]) * (lim[7] + 1), np.int64)   # the rank's view of the region
    val[:] = 255   # never-computed slots hold the largest code: reading one changes the result
    written = np.zeros(len(val), bool)
    for s in range(int(level.max()) + 1):
        kk = keys[level == s]
        if s == 0:
            val[cidx(kk)] = 255   # all heaps empty: LOSS in 0
            written[cidx(kk)] = True
            continue
        pb = box_of_key(kk)
        fills = fill_of[pb]
        best = np.zeros(len(kk), np.int64)
        for i in range(8):
            hi = (kk >> (4 * i)) & 15
            for sub in (1, 2):
                ok = hi >= 1
                child = kk[ok] - (np.minimum(hi[ok], sub) << (4 * i))
                cb = box_of_key(child)
                # a child in the parent's box or in a box this rank computes is read directly;
                # else through the fill code of the heap the step crossed
                cc = np.where((cb != pb[ok]) & ~mine[cb], (fills[ok] >> (3 * i)) & 7, 0)
                src = cidx(bsym_key(cc, child))
                assert written[src].all()
                best[ok] = np.maximum(best[ok], val[src])
        val[cidx(kk)] = (255 - best) + 2 * (best >> 7)
        written[cidx(kk)] = True
    return keys, val[cidx(keys)]


def _record_of_code(c):
    c = np.asarray(c, np.int64)
    return np.where(c >= 128, (1 << 14) | (255 - c), c - 1).astype(np.uint16)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_emulated_rank_solves_match_the_oracle(oracle, world):
    """Each rank, solving only its own boxes and reading the others through the plan's heap
    permutations, gets the C oracle's record for every position of its boxes (root
    0x33337777: 256 boxes, 2^20 positions, every position of them in the root's region)."""
    root = 0x33337777
    ok, orec = oracle.solve(5, (8,), root=root)
    ref = dict(zip(ok.tolist(), orec.tolist()))
    seen = set()
    for r in range(world):
        p = plan(world, r, root)
        keys, val = _emulate_rank(root, world, r, p)
        rec = _record_of_code(val)
        want = np.array([ref[k] for k in keys.tolist()], np.uint16)
        assert np.array_equal(rec, want), r
        own = np.isin(box_of_key(keys), p["own"])
        seen.update(keys[own].tolist())
    assert len(seen) == len(ok)
