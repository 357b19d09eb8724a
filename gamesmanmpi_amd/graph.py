"""Any plugin on the device: explicit-graph solves (GM_GAME_GRAPH).

A plugin that no device descriptor reproduces (``games.identify`` returns None)
is still solved on the GPU: the host walks the plugin itself -- breadth-first
from the root with the reference's four functions (README.md:28-88; the same
expansion as GameState.expand, src/game_state.py:33-41, primitive positions not
expanded, src/new_process.py:120-130) -- numbers every distinct position, and
hands the graph to ``gm_solve_graph``, whose kernels run the retrograde.

Host enumeration is level-synchronous.  A level of at least ``PAR_MIN``
positions is expanded in batches by a pool of worker processes (the plugin's
Python runs in parallel; ``GM_HOST_WORKERS``, default the process's CPU share,
at most 16); the pool is started while the first levels run serially, and the
parent deduplicates each batch's children as it arrives, in level order, so the
numbering is the serial walk's.  Workers rebuild the plugin from its file; when
the caller's module differs from a fresh import in anything that cannot be
passed along (a replaced function, a changed table), the walk stays serial.  Before each level the walk projects the next one from the
growth so far and stops at once -- with the level sizes and the projection in
the message -- when the reachable set would pass ``limit`` positions or the
walk would pass ``budget_s`` seconds: a plugin far too large for host
enumeration (e.g. othello_bit_new.py at its 8x8 default) fails in seconds
instead of running for days.  Positions must be hashable, or numpy arrays
(keyed by dtype, shape and bytes).

Symmetry.  A plugin may declare ``symmetry_functions()``, a list
of ``(function, order)`` pairs (the reference's hook, othello_bit_new.py:224-225,
which its engines never call).  The walk uses those functions that map the root
to itself: the positions reachable from such a root are closed under them, so
it numbers one representative per orbit (the least position of the orbit, in a
fixed byte order), expands only representatives, and counts, exports and
persists every member of every orbit.  A declared function that moves the root
is not used: its images of reachable positions need not be reachable
(Othello's player_flip maps every reachable position to an unreachable one).
"""
import pickle
import importlib.util
import multiprocessing as mp
import os
import time

import numpy as np

from . import _lib

UNDECIDED = 4
PAR_MIN = 1024        # positions in a level before it is expanded by the worker pool
BATCH = 1024          # positions per worker task


class TooLarge(RuntimeError):
    """The plugin's reachable set is projected past the host-enumeration limits."""


def position_key(pos):
    """Hashable identity of a plugin position (numpy boards by dtype/shape/bytes)."""
    if isinstance(pos, np.ndarray):
        return ("ndarray", pos.dtype.str, pos.shape, pos.tobytes())
    return pos


def _order(pos):
    return pickle.dumps(position_key(pos), protocol=4)


def symmetry_generators(module, root):
    """Indices of the plugin's symmetry_functions() that map `root` to itself."""
    decl = getattr(module, "symmetry_functions", None)
    if not callable(decl):
        return []
    out = []
    try:
        items = list(decl())
    except Exception:
        return []
    for i, item in enumerate(items):
        f = item[0] if isinstance(item, tuple) else item
        try:
            if callable(f) and position_key(f(root)) == position_key(root):
                out.append(i)
        except Exception:
            pass
    return out


def _generators(module, idx):
    if not idx:
        return []
    items = list(module.symmetry_functions())
    return [items[i][0] if isinstance(items[i], tuple) else items[i] for i in idx]


def orbit(pos, gens):
    """Every image of pos under the group the functions generate, pos first."""
    out, seen, todo = [pos], {position_key(pos)}, [pos]
    while todo:
        p = todo.pop()
        for g in gens:
            q = g(p)
            k = position_key(q)
            if k not in seen:
                seen.add(k)
                out.append(q)
                todo.append(q)
    return out


def canonical(pos, gens):
    """The orbit's representative: its least member in pickled-key byte order."""
    return min(orbit(pos, gens), key=_order) if gens else pos


def _expand_one(module, pos, gens=()):
    p = module.primitive(pos)
    if not isinstance(p, (int, np.integer)) or not 0 <= int(p) <= 4:
        raise ValueError("primitive(%r) returned %r, not a src.utils code" % (pos, p))
    p = int(p)
    kids = [module.do_move(pos, m) for m in module.gen_moves(pos)] if p == UNDECIDED else []
    if gens:
        kids = [canonical(c, gens) for c in kids]
    return p, kids


# ---------------------------------------------------------------- worker pool
_WORKER_MODULE = None
_WORKER_GENS = []


def _simple(v):
    if isinstance(v, (bool, int, float, str, type(None))):
        return True
    return isinstance(v, tuple) and all(_simple(x) for x in v)


def _load_fresh(path, name="gm_graph_plugin"):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _same(a, b):
    """True when b (a fresh import's attribute) behaves as a (the caller's)."""
    import types
    if a is b:
        return True
    if isinstance(a, types.FunctionType) and isinstance(b, types.FunctionType):
        ca, cb = a.__code__, b.__code__
        if not (ca.co_code == cb.co_code and ca.co_consts == cb.co_consts and ca.co_names == cb.co_names
                and a.__defaults__ == b.__defaults__ and len(a.__closure__ or ()) == len(b.__closure__ or ())):
            return False
        try:   # decorated functions (src.utils encode_int / decode_int): compare what they wrap
            return all(_same(x.cell_contents, y.cell_contents) for x, y in zip(a.__closure__ or (), b.__closure__ or ()))
        except ValueError:   # an empty cell
            return False
    if isinstance(a, types.ModuleType) or isinstance(a, type):
        return a is b or getattr(a, "__name__", 0) == getattr(b, "__name__", 1)
    try:
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return isinstance(a, np.ndarray) and isinstance(b, np.ndarray) and a.dtype == b.dtype and \
                np.array_equal(a, b)
        return type(a) is type(b) and bool(a == b)
    except Exception:
        return False


def _module_spec(module):
    """(file, module-level values) that rebuild the caller's plugin in a worker, or None
    when that cannot be done faithfully.  A value the caller changed is passed along
    if it pickles (ints, tuples, lists, dicts, arrays, ...); a replaced function or
    anything else that differs from the file's own value makes the walk serial --
    a worker would otherwise expand a different game with no error."""
    import pickle
    path = getattr(module, "__file__", None)
    if not path or not os.path.exists(path):
        return None
    try:
        fresh = _load_fresh(path, "gm_graph_plugin_check")
    except Exception:
        return None
    attrs = {}
    for k, v in vars(module).items():
        if k.startswith("__"):
            continue
        if _simple(v):
            attrs[k] = v
        elif hasattr(fresh, k) and _same(v, getattr(fresh, k)):
            continue
        else:
            import types
            if isinstance(v, (types.FunctionType, types.ModuleType, type)):
                return None
            try:
                pickle.dumps(v)
            except Exception:
                return None
            attrs[k] = v
    return path, attrs


def _worker_init(path, attrs, gen_idx=()):
    global _WORKER_MODULE, _WORKER_GENS
    mod = _load_fresh(path)
    for k, v in attrs.items():   # values the caller set on its module (board size, ...)
        setattr(mod, k, v)
    _WORKER_MODULE = mod
    _WORKER_GENS = _generators(mod, list(gen_idx))


def _worker_expand(batch):
    return [_expand_one(_WORKER_MODULE, pos, _WORKER_GENS) for pos in batch]


def _default_workers():
    """GM_HOST_WORKERS, else the CPUs this process may use (the GPU box grants each GPU a
    share of a large machine and says so in OMP_NUM_THREADS), at most 16."""
    env = os.environ.get("GM_HOST_WORKERS")
    if env:
        return max(1, int(env))
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(16, n))


def _noop():
    return 0


def _main_importable():
    """Spawned workers re-import the parent's __main__; a script from stdin cannot be."""
    import sys
    main = sys.modules.get("__main__")
    path = getattr(main, "__file__", None)
    return path is None or os.path.exists(path)


class _Expander:
    """Expands a level serially or, when large, in batches on a spawned worker pool,
    yielding (primitive, children) per position in level order as batches complete.
    The pool starts at construction (its processes import while the small first
    levels run serially).  A pool failure (a worker that cannot start or dies)
    before any result of a level was yielded falls back to the serial walk."""

    def __init__(self, module, workers, gen_idx=()):
        self.module = module
        self.workers = workers
        self.gens = _generators(module, list(gen_idx))
        self.pool = None
        self.spec = _module_spec(module) if workers > 1 and _main_importable() else None
        if self.spec is not None:
            from concurrent.futures import ProcessPoolExecutor
            try:
                self.pool = ProcessPoolExecutor(self.workers, mp_context=mp.get_context("spawn"),
                                                initializer=_worker_init, initargs=self.spec + (tuple(gen_idx),))
                for _ in range(self.workers):   # start every worker now
                    self.pool.submit(_noop)
            except (OSError, ImportError):
                self.close()
                self.spec = None

    def __call__(self, level):
        if self.spec is None or len(level) < PAR_MIN:
            for pos in level:
                yield _expand_one(self.module, pos, self.gens)
            return
        from concurrent.futures.process import BrokenProcessPool
        batches = [level[i:i + BATCH] for i in range(0, len(level), BATCH)]
        done = 0
        try:
            for res in self.pool.map(_worker_expand, batches):
                for r in res:
                    yield r
                done += 1
        except (BrokenProcessPool, OSError, ImportError):
            if done:
                raise
            self.close()
            self.spec = None
            for pos in level:
                yield _expand_one(self.module, pos, self.gens)

    def close(self):
        if self.pool is not None:
            self.pool.shutdown(wait=True, cancel_futures=True)
            self.pool = None


def enumerate_graph(module, root, limit=50_000_000, workers=None, budget_s=3600.0, symmetry=()):
    """Positions reachable from ``root`` (index 0) with primitive codes and CSR children.

    ``symmetry``: indices of ``symmetry_functions()`` that fix the root
    (symmetry_generators); the positions are then the orbit representatives.
    Raises TooLarge as soon as the projected next level would pass ``limit``
    positions or the walk's projected time would pass ``budget_s`` seconds."""
    workers = _default_workers() if workers is None else max(1, int(workers))
    root = canonical(root, _generators(module, list(symmetry)))
    index = {position_key(root): 0}
    positions = [root]
    prim = []
    off = [0]
    kids = []
    sizes = []
    level = [root]
    expand = _Expander(module, workers, symmetry)
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
    """Keys of a graph solve are position indices -- of orbit representatives when the
    plugin declares symmetries that fix the root; ``pos`` maps a key back to its
    representative and ``members`` to every position it stands for."""
    game_id = _lib.GAME_GRAPH
    params = ()
    name = "graph"

    def __init__(self, module, root, workers=None, symmetry=None):
        self.module = module
        self.symmetry = symmetry_generators(module, root) if symmetry is None else list(symmetry)
        self.gens = _generators(module, self.symmetry)
        self.positions, self.prim, self.off, self.kids = enumerate_graph(module, root, workers=workers,
                                                                         symmetry=self.symmetry)
        self._index = {position_key(p): i for i, p in enumerate(self.positions)}
        self.n_positions = (sum(len(orbit(p, self.gens)) for p in self.positions) if self.gens
                            else len(self.positions))

    def key(self, pos):
        try:
            return self._index[position_key(canonical(pos, self.gens))]
        except KeyError:
            raise ValueError("position not reachable from the root") from None

    def pos(self, key):
        return self.positions[int(key)]

    def members(self, key):
        """The reachable positions key stands for (its orbit; just pos(key) without symmetry)."""
        p = self.positions[int(key)]
        return orbit(p, self.gens) if self.gens else [p]
