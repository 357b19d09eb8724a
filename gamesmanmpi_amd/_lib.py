"""ctypes binding of libgmsolve.so (include/gmsolve.h).

The library is built in-tree (``python -m gamesmanmpi_amd.build``).  There is no
fallback: if the library is missing or cannot be loaded, importing the solver
raises, so a GPU run can never silently use some other code path.
"""
import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# GM_LIB_PATH: development aid to load an experimental build of the same library
LIB_PATH = os.environ.get("GM_LIB_PATH") or os.path.join(PKG, "libgmsolve.so")

GAME_FOUR_TO_ONE, GAME_TTT, GAME_TOOT, GAME_OTHELLO, GAME_SUBTRACT, GAME_GRAPH = 1, 2, 3, 4, 5, 6
ENGINE_AUTO, ENGINE_DENSE, ENGINE_SPARSE, ENGINE_DIST_DENSE, ENGINE_DIST_SPARSE, ENGINE_GRAPH = 0, 1, 2, 3, 4, 5
OPT_ENGINE, OPT_SUB_LOW, OPT_GRAPH, OPT_TIMING, OPT_VIRTUAL_RANKS, OPT_SUB_THREADS = 1, 2, 3, 4, 5, 6
OPT_SUB_INTERLEAVE = 7
OPT_SUB_ORDER = 8
OPT_DIST_BATCH = 9
OPT_DIST_SLOTS = 10
OPT_DIST_SYMMETRY = 11
OPT_DIST_SOLO = 12
OPT_DIST_OWNER = 13
OPT_SYMMETRY = 14
OPT_BOX_FLOW = 15
OPT_BOX_SPLIT = 16
OPT_BOX_TRANSPORT = 17
OPT_SPARSE_TRANSPORT = 18
OPT_POISON = 19
ABI_VERSION = 2
BUF_DENSE_TABLE = 1
PLAN_SHAPE, PLAN_OWN, PLAN_FILL, PLAN_SEND, PLAN_RECV, PLAN_OPS, PLAN_XDEST = 0, 1, 2, 3, 4, 5, 6
BOXPLAN_SHAPE, BOXPLAN_BOXES, BOXPLAN_FILLS, BOXPLAN_TIER_OFF, BOXPLAN_OWN = 0, 1, 2, 3, 4
BOXPLAN_SEND, BOXPLAN_SEND_OFF, BOXPLAN_RECV, BOXPLAN_RECV_OFF, BOXPLAN_HALO, BOXPLAN_OPS = 5, 6, 7, 8, 9, 10
BOXPLAN_COUNTS, BOXPLAN_SRCS, BOXPLAN_DSTS = 11, 12, 13
BOP_TIER, BOP_PACK, BOP_UNPACK, BOP_SEND, BOP_RECV, BOP_RECORD, BOP_WAIT = range(7)
BEV_DONE, BEV_PACKED = range(2)
REC_UNSOLVED = 0xFFFF

ERRORS = {
    -1: "GM_E_ARG", -2: "GM_E_GAME", -3: "GM_E_HIP", -4: "GM_E_NOMEM", -5: "GM_E_STATE",
    -6: "GM_E_DRAW", -7: "GM_E_NOMOVES", -8: "GM_E_CAP", -9: "GM_E_COMM", -10: "GM_E_KEY",
}

# Every symbol include/gmsolve.h declares (tests check the library exports them).
SYMBOLS = ("gm_version", "gm_last_error", "gm_device_count", "gm_open", "gm_set_stream",
           "gm_set_option", "gm_pack_initial", "gm_expand_host", "gm_comm_unique_id",
           "gm_set_comm", "gm_solve", "gm_solve_graph", "gm_export", "gm_query", "gm_digest", "gm_stats",
           "gm_tier_counts", "gm_adopt_buffer", "gm_dense_table", "gm_dist_plan", "gm_box_plan",
           "gm_rank_stats", "gm_rank_op_ms", "gm_close", "gm_key_words", "gm_pack_initial_key",
           "gm_expand_host_key", "gm_solve_key", "gm_export_key", "gm_query_key", "gm_sparse_layout")


class GMError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "GM_E?"), code, message))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ("n_positions", ctypes.c_uint64),
        ("n_primitive", ctypes.c_uint64),
        ("n_tiers", ctypes.c_int32),
        ("world", ctypes.c_int32),
        ("solve_ms", ctypes.c_double),
        ("forward_ms", ctypes.c_double),
        ("backward_ms", ctypes.c_double),
        ("exchange_ms", ctypes.c_double),
        ("algo_bytes", ctypes.c_uint64),
        ("table_bytes", ctypes.c_uint64),
        ("exchanged_bytes", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("kernel_launches", ctypes.c_int32),
        ("engine", ctypes.c_int32),
        ("n_edges", ctypes.c_uint64),
        ("flow_fallbacks", ctypes.c_int32),
        ("n_stored", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


_lib = None


def lib():
    """Load libgmsolve.so once; raise loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libgmsolve.so is not built (%s); run `python -m gamesmanmpi_amd.build`"
                           % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    u64, i32, i64 = ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    sig = {
        "gm_version": (ctypes.c_int, []),
        "gm_last_error": (ctypes.c_char_p, []),
        "gm_device_count": (ctypes.c_int, []),
        "gm_open": (ctypes.c_int, [ctypes.c_int, P(i32), ctypes.c_int, ctypes.c_int, P(vp)]),
        "gm_set_stream": (ctypes.c_int, [vp, vp]),
        "gm_set_option": (ctypes.c_int, [vp, ctypes.c_int, i64]),
        "gm_pack_initial": (ctypes.c_int, [vp, P(u64)]),
        "gm_expand_host": (ctypes.c_int, [vp, u64, P(u64), ctypes.c_int, P(ctypes.c_int),
                                          P(ctypes.c_int), P(i64)]),
        "gm_comm_unique_id": (ctypes.c_int, [vp, ctypes.c_int]),
        "gm_set_comm": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int]),
        "gm_solve": (ctypes.c_int, [vp, u64, P(u64), P(ctypes.c_uint16)]),
        "gm_solve_graph": (ctypes.c_int, [vp, u64, vp, vp, vp, P(ctypes.c_uint16)]),
        "gm_export": (ctypes.c_int, [vp, vp, vp, u64, P(u64)]),
        "gm_query": (ctypes.c_int, [vp, vp, vp, u64]),
        "gm_digest": (ctypes.c_int, [vp, P(u64), P(u64)]),
        "gm_stats": (ctypes.c_int, [vp, P(Stats)]),
        "gm_tier_counts": (ctypes.c_int, [vp, vp, ctypes.c_int, P(ctypes.c_int)]),
        "gm_adopt_buffer": (ctypes.c_int, [vp, ctypes.c_int, vp, u64]),
        "gm_dense_table": (ctypes.c_int, [vp, P(vp), P(u64)]),
        "gm_dist_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int,
                                        vp, u64, P(u64), vp, u64, P(u64)]),
        "gm_box_plan": (ctypes.c_int, [u64, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, vp, u64,
                                       P(u64)]),
        "gm_rank_stats": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, P(ctypes.c_int)]),
        "gm_rank_op_ms": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, P(ctypes.c_int)]),
        "gm_close": (None, [vp]),
        "gm_key_words": (ctypes.c_int, [vp]),
        "gm_pack_initial_key": (ctypes.c_int, [vp, vp]),
        "gm_expand_host_key": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int), P(i64)]),
        "gm_solve_key": (ctypes.c_int, [vp, vp, P(u64), P(ctypes.c_uint16)]),
        "gm_export_key": (ctypes.c_int, [vp, vp, vp, u64, P(u64)]),
        "gm_query_key": (ctypes.c_int, [vp, vp, vp, u64]),
        "gm_sparse_layout": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().gm_last_error()
        raise GMError(rc, msg.decode() if msg else "")
    return rc


def dist_plan(heaps, world, rank, what, axis=0, batch=4, slots=4, symmetry=1, owner=0):
    """gm_dist_plan -> (off, data) as uint32 numpy arrays (host only, no GPU)."""
    import numpy as np
    L = lib()
    opts = (ctypes.c_int32 * 3)(batch, slots, symmetry | owner << 1)
    n_off, n_data = ctypes.c_uint64(), ctypes.c_uint64()
    check(L.gm_dist_plan(heaps, world, rank, opts, what, axis, None, 0, ctypes.byref(n_off), None, 0,
                         ctypes.byref(n_data)))
    off = np.zeros(max(1, n_off.value), dtype=np.uint32)
    data = np.zeros(max(1, n_data.value), dtype=np.uint32)
    check(L.gm_dist_plan(heaps, world, rank, opts, what, axis, off.ctypes.data, len(off), ctypes.byref(n_off),
                         data.ctypes.data, len(data), ctypes.byref(n_data)))
    return off[:n_off.value], data[:n_data.value]


def box_plan(world, rank, what, root=0xFFFFFFFF, axis=0, batch=4, symmetry=1, split=0, loopback=0, transport=0):
    """gm_box_plan -> uint32 numpy array (host only, no GPU): rank `rank`'s part of the split
    box solve (csrc/dist_box.hip).  batch / symmetry / split / transport: GM_OPT_DIST_BATCH,
    GM_OPT_DIST_SYMMETRY, GM_OPT_BOX_SPLIT, GM_OPT_BOX_TRANSPORT; loopback: the op list of a
    virtual rank."""
    import numpy as np
    L = lib()
    opts = (ctypes.c_int32 * 5)(batch, symmetry, split, loopback, transport)
    n = ctypes.c_uint64()
    check(L.gm_box_plan(root, world, rank, opts, what, axis, None, 0, ctypes.byref(n)))
    out = np.zeros(max(1, n.value), dtype=np.uint32)
    check(L.gm_box_plan(root, world, rank, opts, what, axis, out.ctypes.data, len(out), ctypes.byref(n)))
    return out[:n.value]


def int_to_words(key, nwords):
    """A key (Python int) as `nwords` u64 words, least significant first (include/gmsolve.h)."""
    return [(int(key) >> (64 * i)) & ((1 << 64) - 1) for i in range(nwords)]


def words_to_int(words):
    """u64 key words (least significant first) -> one Python int."""
    return sum(int(w) << (64 * i) for i, w in enumerate(words))


def sparse_layout(world, steps, counts, rank):
    """gm_sparse_layout (host only): (seg, send_off, recv_off, recv_seg) of rank `rank` for the
    world x (world * steps) count matrix of one exchange of the hash-sharded sparse engine."""
    import numpy as np
    m = np.ascontiguousarray(counts, dtype=np.uint64).reshape(world, world * steps)
    seg = np.zeros(world * steps, dtype=np.uint64)
    so = np.zeros(world + 1, dtype=np.uint64)
    ro = np.zeros(world + 1, dtype=np.uint64)
    rs = np.zeros(world * steps, dtype=np.uint64)
    check(lib().gm_sparse_layout(world, steps, m.ctypes.data, rank, seg.ctypes.data, so.ctypes.data, ro.ctypes.data,
                                 rs.ctypes.data))
    return seg, so, ro, rs
