"""Any plugin on the device: explicit-graph solves (GM_GAME_GRAPH).

A plugin that no device descriptor reproduces (``games.identify`` returns None)
is still solved on the GPU: the host walks the plugin itself -- breadth-first
from the root with the reference's four functions (README.md:28-88; the same
expansion as GameState.expand, src/game_state.py:33-41, primitive positions not
expanded, src/new_process.py:120-130) -- numbers every distinct position, and
hands the graph to ``gm_solve_graph``, whose kernels run the retrograde.

Host enumeration is level-synchronous.  A level of at least ``PAR_MIN``
positions is expanded in batches by a pool of worker processes (the plugin's
Python runs in parallel; ``GM_HOST_WORKERS``, default min(8, cpus)); the parent
deduplicates the returned children in level order, so the numbering is the
serial walk's.  Before each level the walk projects the next one from the
growth so far and stops at once -- with the level sizes and the projection in
the message -- when the reachable set would pass ``limit`` positions or the
walk would pass ``budget_s`` seconds: a plugin far too large for host
enumeration (e.g. othello_bit_new.py at its 8x8 default) fails in seconds
instead of running for days.  Positions must be hashable, or numpy arrays
(keyed by dtype, shape and bytes).
"""
import importlib.util
import multiprocessing as mp
import os
import time

import numpy as np

from . import _lib

UNDECIDED = 4
PAR_MIN = 4096        # positions in a level before it is expanded by the worker pool
BATCH = 2048          # positions per worker task


class TooLarge(RuntimeError):
    """The plugin's reachable set is projected past the host-enumeration limits."""


def position_key(pos):
    """Hashable identity of a plugin position (numpy boards by dtype/shape/bytes)."""
    if isinstance(pos, np.ndarray):
        return ("ndarray", pos.dtype.str, pos.shape, pos.tobytes())
    return pos


def _expand_one(module, pos):
    p = module.primitive(pos)
    if not isinstance(p, (int, np.integer)) or not 0 <= int(p) <= 4:
        raise ValueError("primitive(%r) returned %r, not a src.utils code" % (pos, p))
    p = int(p)
    kids = [module.do_move(pos, m) for m in module.gen_moves(pos)] if p == UNDECIDED else []
    return p, kids


# ---------------------------------------------------------------- worker pool
_WORKER_MODULE = None


def _simple(v):
    if isinstance(v, (bool, int, float, str, type(None))):
        return True
    return isinstance(v, tuple) and all(_simple(x) for x in v)


def _module_spec(module):
    """(file, simple module-level values) that rebuild the plugin in a worker, or None."""
    path = getattr(module, "__file__", None)
    if not path or not os.path.exists(path):
        return None
    attrs = {k: v for k, v in vars(module).items() if not k.startswith("__") and _simple(v)}
    return path, attrs


def _worker_init(path, attrs):
    global _WORKER_MODULE
    spec = importlib.util.spec_from_file_location("gm_graph_plugin", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for k, v in attrs.items():   # parameters the caller set on its module (board size, ...)
        setattr(mod, k, v)
    _WORKER_MODULE = mod


def _worker_expand(batch):
    return [_expand_one(_WORKER_MODULE, pos) for pos in batch]


def _default_workers():
    env = os.environ.get("GM_HOST_WORKERS")
    if env:
        return max(1, int(env))
    return max(1, min(8, os.cpu_count() or 1))


def _main_importable():
    """Spawned workers re-import the parent's __main__; a script from stdin cannot be."""
    import sys
    main = sys.modules.get("__main__")
    path = getattr(main, "__file__", None)
    return path is None or os.path.exists(path)


class _Expander:
    """Expands a level serially or, when large, in batches on a spawned worker pool.
    Any pool failure (a worker that cannot start or dies) falls back to the serial walk."""

    def __init__(self, module, workers):
        self.module = module
        self.workers = workers
        self.pool = None
        self.spec = _module_spec(module) if workers > 1 and _main_importable() else None

    def __call__(self, level):
        if self.spec is None or len(level) < PAR_MIN:
            return [_expand_one(self.module, pos) for pos in level]
        from concurrent.futures import ProcessPoolExecutor
        from concurrent.futures.process import BrokenProcessPool
        try:
            if self.pool is None:
                self.pool = ProcessPoolExecutor(self.workers, mp_context=mp.get_context("spawn"),
                                                initializer=_worker_init, initargs=self.spec)
            batches = [level[i:i + BATCH] for i in range(0, len(level), BATCH)]
            out = []
            for res in self.pool.map(_worker_expand, batches):
                out.extend(res)
            return out
        except (BrokenProcessPool, OSError, ImportError):
            self.close()
            self.spec = None
            return [_expand_one(self.module, pos) for pos in level]

    def close(self):
        if self.pool is not None:
            self.pool.shutdown(wait=True, cancel_futures=True)
            self.pool = None


def enumerate_graph(module, root, limit=50_000_000, workers=None, budget_s=3600.0):
    """Positions reachable from ``root`` (index 0) with primitive codes and CSR children.

    Raises TooLarge as soon as the projected next level would pass ``limit``
    positions or the walk's projected time would pass ``budget_s`` seconds."""
    workers = _default_workers() if workers is None else max(1, int(workers))
    index = {position_key(root): 0}
    positions = [root]
    prim = []
    off = [0]
    kids = []
    sizes = []
    level = [root]
    expand = _Expander(module, workers)
    t0 = time.perf_counter()
    try:
        while level:
            tl = time.perf_counter()
            sizes.append(len(level))
            nxt = []
            for p, children in expand(level):
                prim.append(p)
                for child in children:
                    k = position_key(child)
                    j = index.get(k)
                    if j is None:
                        j = len(positions)
                        if j >= limit:
                            raise TooLarge("more than %d positions: too large for host enumeration (levels %s)"
                                           % (limit, sizes))
                        index[k] = j
                        positions.append(child)
                        nxt.append(child)
                    kids.append(j)
                off.append(len(kids))
            # fail fast: project the level after this one from the last growth factor
            if nxt and len(level) > 0:
                growth = len(nxt) / len(level)
                projected = len(positions) + len(nxt) * growth
                dt = time.perf_counter() - tl
                elapsed = time.perf_counter() - t0
                if projected > limit or (growth > 1 and elapsed + dt * growth * growth > budget_s):
                    raise TooLarge(
                        "plugin %s: after %d levels (sizes %s, %d positions, %.1f s) the next level is "
                        "projected at ~%.3g positions (growth x%.2f per level): past the host-enumeration "
                        "limits (%d positions, %.0f s); no device descriptor reproduces this plugin at these "
                        "parameters" % (getattr(module, "__name__", module), len(sizes), sizes + [len(nxt)],
                                        len(positions), elapsed, len(nxt) * growth, growth, limit, budget_s))
            level = nxt
    finally:
        expand.close()
    return positions, np.array(prim, dtype=np.uint8), np.array(off, dtype=np.uint64), np.array(kids, dtype=np.uint32)


class GraphCodec:
    """Keys of a graph solve are position indices; ``pos`` maps them back."""
    game_id = _lib.GAME_GRAPH
    params = ()
    name = "graph"

    def __init__(self, module, root, workers=None):
        self.module = module
        self.positions, self.prim, self.off, self.kids = enumerate_graph(module, root, workers=workers)
        self._index = {position_key(p): i for i, p in enumerate(self.positions)}

    def key(self, pos):
        try:
            return self._index[position_key(pos)]
        except KeyError:
            raise ValueError("position not reachable from the root") from None

    def pos(self, key):
        return self.positions[int(key)]
