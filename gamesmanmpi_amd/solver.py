"""Host-side solver API: the drop-in for the reference's Process/Job engine.

``Solver(module)`` plays the role of ``Process`` + ``GameState``
(reference src/new_process.py:62-94, src/game_state.py): it binds a plugin
module to a device descriptor, solves every position reachable from the root
in one ``gm_solve`` call, and answers lookups (the reference's
``resolved``/``remote`` tables, src/new_process.py:76-78).
"""
import ctypes
import os

import numpy as np

from . import _lib, games
from .src_utils import to_str

WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4


def split_record(rec):
    """u16 record -> (value, remoteness); (None, None) for 0xFFFF."""
    rec = int(rec)
    if rec == _lib.REC_UNSOLVED:
        return None, None
    return rec >> 14, rec & 0x3FFF


class NoDescriptor(RuntimeError):
    pass


class Context:
    """Thin RAII wrapper over one ``gm_ctx``."""

    def __init__(self, game_id, params=(), device=-1):
        self.L = _lib.lib()
        arr = (ctypes.c_int32 * max(1, len(params)))(*params)
        h = ctypes.c_void_p()
        _lib.check(self.L.gm_open(game_id, arr, len(params), device, ctypes.byref(h)))
        self.h = h
        self.game_id = game_id
        self.params = tuple(params)
        # u64 words per key: 1, or 3 for boards past 64 bits (Othello 8x8); keys are then Python
        # ints on the host and (n, words) uint64 arrays in bulk (gm_*_key)
        self.words = self.L.gm_key_words(h)

    def set_option(self, opt, value):
        _lib.check(self.L.gm_set_option(self.h, opt, int(value)))

    def set_stream(self, stream_ptr):
        _lib.check(self.L.gm_set_stream(self.h, ctypes.c_void_p(stream_ptr or 0)))

    def set_comm(self, rank, world, uid=None):
        buf = ctypes.create_string_buffer(uid, 128) if uid is not None else None
        _lib.check(self.L.gm_set_comm(self.h, rank, world, buf, 128 if buf is not None else 0))

    def initial(self):
        if self.words > 1:
            w = (ctypes.c_uint64 * self.words)()
            _lib.check(self.L.gm_pack_initial_key(self.h, w))
            return _lib.words_to_int(w)
        k = ctypes.c_uint64()
        _lib.check(self.L.gm_pack_initial(self.h, ctypes.byref(k)))
        return k.value

    def solve(self, root):
        n = ctypes.c_uint64()
        r = ctypes.c_uint16()
        if self.words > 1:
            w = (ctypes.c_uint64 * self.words)(*_lib.int_to_words(root, self.words))
            _lib.check(self.L.gm_solve_key(self.h, w, ctypes.byref(n), ctypes.byref(r)))
        else:
            _lib.check(self.L.gm_solve(self.h, root, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    def key_array(self, keys):
        """Keys (Python ints, or an (n, words) uint64 array) -> the array gm_query_key takes."""
        if self.words == 1:
            return np.ascontiguousarray(keys, dtype=np.uint64)
        a = np.asarray(keys) if not isinstance(keys, list) else None
        if a is not None and a.dtype == np.uint64 and a.ndim == 2:
            return np.ascontiguousarray(a)
        return np.array([_lib.int_to_words(k, self.words) for k in keys], dtype=np.uint64).reshape(-1, self.words)

    def solve_graph(self, prim, off, kids):
        """gm_solve_graph over an explicit graph (gamesmanmpi_amd/graph.py)."""
        import numpy as np
        prim = np.ascontiguousarray(prim, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        kids = np.ascontiguousarray(kids, dtype=np.uint32)
        r = ctypes.c_uint16()
        _lib.check(self.L.gm_solve_graph(self.h, len(prim), prim.ctypes.data, off.ctypes.data,
                                         kids.ctypes.data if len(kids) else None, ctypes.byref(r)))
        return len(prim), r.value

    def export(self):
        """Sorted keys and records (multi-word keys: an (n, words) uint64 array)."""
        n = ctypes.c_uint64()
        if self.words > 1:
            _lib.check(self.L.gm_export_key(self.h, None, None, 0, ctypes.byref(n)))
            keys = np.empty((n.value, self.words), dtype=np.uint64)
            recs = np.empty(n.value, dtype=np.uint16)
            _lib.check(self.L.gm_export_key(self.h, keys.ctypes.data, recs.ctypes.data, n.value, ctypes.byref(n)))
            return keys[:n.value], recs[:n.value]
        _lib.check(self.L.gm_export(self.h, None, None, 0, ctypes.byref(n)))
        keys = np.empty(n.value, dtype=np.uint64)
        recs = np.empty(n.value, dtype=np.uint16)
        _lib.check(self.L.gm_export(self.h, keys.ctypes.data, recs.ctypes.data, n.value, ctypes.byref(n)))
        return keys[:n.value], recs[:n.value]

    def query(self, keys):
        keys = self.key_array(keys)
        out = np.empty(len(keys), dtype=np.uint16)
        if self.words > 1:
            _lib.check(self.L.gm_query_key(self.h, keys.ctypes.data, out.ctypes.data, len(keys)))
        else:
            _lib.check(self.L.gm_query(self.h, keys.ctypes.data, out.ctypes.data, len(keys)))
        return out

    def digest(self):
        d, n = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self.L.gm_digest(self.h, ctypes.byref(d), ctypes.byref(n)))
        return d.value, n.value

    def stats(self):
        s = _lib.Stats()
        _lib.check(self.L.gm_stats(self.h, ctypes.byref(s)))
        return s.as_dict()

    def tier_counts(self):
        n = ctypes.c_int()
        _lib.check(self.L.gm_tier_counts(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(max(1, n.value), dtype=np.uint64)
        _lib.check(self.L.gm_tier_counts(self.h, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value]

    def rank_stats(self):
        """Per rank of the last split box solve (gm_rank_stats): GPU ms from its first tier launch
        to its last (GM_OPT_TIMING), boxes computed, halo bytes received per solve."""
        n = ctypes.c_int()
        _lib.check(self.L.gm_rank_stats(self.h, None, None, None, 0, ctypes.byref(n)))
        ms = np.zeros(max(1, n.value), dtype=np.float64)
        boxes = np.zeros(max(1, n.value), dtype=np.uint64)
        recv = np.zeros(max(1, n.value), dtype=np.uint64)
        _lib.check(self.L.gm_rank_stats(self.h, ms.ctypes.data, boxes.ctypes.data, recv.ctypes.data, n.value,
                                        ctypes.byref(n)))
        return [{"kernel_ms": float(ms[i]), "boxes": int(boxes[i]), "recv_bytes": int(recv[i])}
                for i in range(n.value)]

    def rank_op_ms(self, rank):
        """GPU ms of every op of `rank`'s op list in the last split box solve (GM_OPT_TIMING)."""
        n = ctypes.c_int()
        _lib.check(self.L.gm_rank_op_ms(self.h, rank, None, 0, ctypes.byref(n)))
        out = np.zeros(max(1, n.value), dtype=np.float64)
        _lib.check(self.L.gm_rank_op_ms(self.h, rank, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value]

    def adopt_dense_table(self, dev_ptr, nbytes):
        _lib.check(self.L.gm_adopt_buffer(self.h, _lib.BUF_DENSE_TABLE, ctypes.c_void_p(dev_ptr), nbytes))

    def dense_table(self):
        p, b = ctypes.c_void_p(), ctypes.c_uint64()
        _lib.check(self.L.gm_dense_table(self.h, ctypes.byref(p), ctypes.byref(b)))
        return p.value, b.value

    def close(self):
        if getattr(self, "h", None):
            self.L.gm_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Solver:
    """Strong-solve a plugin module on the GPU.

    ``module`` is a GamesmanMPI plugin; ``root`` defaults to
    ``module.initial_position()`` (GameState.INITIAL_POS, src/game_state.py:15).
    A plugin that no device descriptor reproduces is solved as an explicit graph
    (gamesmanmpi_amd/graph.py): the host enumerates it with the plugin's own
    functions and the device resolves it; ``graph=True`` forces that path,
    ``graph=False`` raises NoDescriptor instead.
    """

    def __init__(self, module, root=None, device=-1, engine=None, codec=None, graph=None):
        self.module = module
        self.root = module.initial_position() if root is None else root
        if codec is None and not graph:
            codec = games.identify(module, self.root)
        if codec is None:
            if graph is False:
                raise NoDescriptor(
                    "no device descriptor reproduces plugin %r; supported: Four-To-One, "
                    "tic-tac-toe (mttt / numpy), Toot-and-Otto and Othello bitboards, "
                    "the subtraction game" % getattr(module, "__file__", module))
            from .graph import GraphCodec
            codec = GraphCodec(module, self.root)
        self.codec = codec
        self.ctx = Context(self.codec.game_id, self.codec.params, device)
        if engine is not None:
            self.ctx.set_option(_lib.OPT_ENGINE, engine)
        self.root_key = self.codec.key(self.root)
        self.n_positions = None
        self.root_record = None

    def solve(self):
        if self.codec.game_id == _lib.GAME_GRAPH:
            c = self.codec
            _, self.root_record = self.ctx.solve_graph(c.prim, c.off, c.kids)
            self.n_positions = c.n_positions   # every orbit member (gamesmanmpi_amd/graph.py)
        else:
            self.n_positions, self.root_record = self.ctx.solve(self.root_key)
        return self.n_positions, self.root_record

    @property
    def value(self):
        return split_record(self.root_record)[0]

    @property
    def remoteness(self):
        return split_record(self.root_record)[1]

    def root_line(self):
        """The reference's root line (src/new_process.py:47-52)."""
        v, r = split_record(self.root_record)
        return "%s in %d moves" % (to_str(v), r)

    def lookup(self, pos):
        rec = self.ctx.query([self.codec.key(pos)])[0]
        return split_record(rec)

    def table(self):
        """Sorted keys and u16 records of every solved position."""
        return self.ctx.export()

    def close(self):
        self.ctx.close()


def dump_table(path, keys, records, meta=None):
    """Write a solved table as ``.npz`` (sorted u64 keys, u16 records)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    np.savez(path, keys=keys, records=records, meta=str(meta or {}))
