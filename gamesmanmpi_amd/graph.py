"""Any plugin on the device: explicit-graph solves (GM_GAME_GRAPH).

A plugin that no device descriptor reproduces (``games.identify`` returns None)
is still solved on the GPU: the host walks the plugin itself -- breadth-first
from the root with the reference's four functions (README.md:28-88; the same
expansion as GameState.expand, src/game_state.py:33-41, primitive positions not
expanded, src/new_process.py:120-130) -- numbers every distinct position, and
hands the graph to ``gm_solve_graph``, whose kernels run the retrograde.

Host enumeration is breadth-first.  Once the graph is projected past a few
thousand positions, worker processes take over (``GM_HOST_WORKERS``, default the
process's CPU share, at most 16; walk_worker.py): each owns the positions whose
fingerprint maps to it, expands its frontier, sends every child to the child's
owner and keeps the new ones, and the parent numbers each level from the workers'
fingerprint reports, so the numbering is the serial walk's.  Workers rebuild the
plugin from its file; when the caller's module differs from a fresh import in
anything that cannot be passed along (a replaced function, a changed table), the
walk stays serial.  Before each level the walk projects the next one from the
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
import multiprocessing as mp
import os
import time

import numpy as np

from . import _lib
from .walk_worker import (_order, canonical, expand_one as _expand_one, fingerprint as _fingerprint,  # noqa: F401
                          generators as _generators, load_fresh as _load_fresh, orbit, owner as _owner,
                          position_key, worker_main)

UNDECIDED = 4
PAR_MIN = 2048        # positions in a level before the walk goes parallel
PAR_START = 8192      # positions so far + the projected next level (or twice that level) that start the
                      # worker processes


def _halves(F):
    """(first 8 bytes, last 8 bytes) of 16-byte fingerprints as big-endian u64, so that the
    pair orders like the bytes."""
    w = np.frombuffer(np.ascontiguousarray(F).tobytes(), dtype=">u8")
    return w[0::2].astype(np.uint64), w[1::2].astype(np.uint64)


class TooLarge(RuntimeError):
    """The plugin's reachable set is projected past the host-enumeration limits."""


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


# ---------------------------------------------------------------- worker pool

def _simple(v):
    if isinstance(v, (bool, int, float, str, type(None))):
        return True
    return isinstance(v, tuple) and all(_simple(x) for x in v)


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


def _main_importable():
    """Spawned workers re-import the parent's __main__; a script from stdin cannot be."""
    import sys
    main = sys.modules.get("__main__")
    path = getattr(main, "__file__", None)
    return path is None or os.path.exists(path)


def _start_method():
    """forkserver where the platform has it (workers fork from a clean server process that
    has imported walk_worker: ~10 ms to start them instead of ~50 ms of interpreter start
    each), else spawn.  Never fork: the caller may hold a GPU context.  GM_GRAPH_START
    overrides."""
    m = os.environ.get("GM_GRAPH_START")
    if m:
        return m
    return "forkserver" if "forkserver" in mp.get_all_start_methods() else "spawn"


def _prestart():
    """Start the fork server ahead of the workers (it imports in the background)."""
    if _start_method() != "forkserver":
        return
    import multiprocessing.forkserver as fs
    ctx = mp.get_context("forkserver")
    ctx.set_forkserver_preload(["gamesmanmpi_amd.walk_worker"])
    fs.ensure_running()


class _ShardPool:
    """The parallel walk's worker processes (forkserver or spawn): one pipe each to the
    parent; the workers connect to each other themselves (walk_worker._mesh)."""

    def __init__(self, spec, nw, gen_idx):
        ctx = mp.get_context(_start_method())
        self.nw = nw
        self.conns, self.procs = [], []
        tag = "gm-walk-%d-%d-%s" % (os.getpid(), id(self), os.urandom(4).hex())
        key = os.urandom(32)   # authenticates the workers' mesh connections (walk_worker._mesh)
        self.start_s = []
        self.t_start = time.time()
        for w in range(nw):
            t = time.perf_counter()
            a, b = ctx.Pipe()
            pr = ctx.Process(target=worker_main, args=(b, w, nw, tag, key, spec[0], spec[1], tuple(gen_idx)),
                             daemon=True)
            pr.start()
            b.close()
            self.conns.append(a)
            self.procs.append(pr)
            self.start_s.append(time.perf_counter() - t)
        self.ready = False
        self.ready_at = []

    def recv(self, w, *kinds):
        try:
            msg = self.conns[w].recv()
        except EOFError:
            raise RuntimeError("graph walk worker %d exited unexpectedly (exit code %s)"
                               % (w, self.procs[w].exitcode)) from None
        if msg[0] == "error":
            raise RuntimeError("graph walk worker %d failed:\n%s" % (w, msg[1]))
        assert msg[0] in kinds, msg[0]
        return msg

    def wait_ready(self):
        if not self.ready:
            for w in range(self.nw):
                self.ready_at.append(self.recv(w, "ready")[1] - self.t_start)
            self.ready = True

    def poll_ready(self):
        """True once every worker has imported the plugin (does not block)."""
        if not self.ready and all(c.poll() for c in self.conns):
            self.wait_ready()
        return self.ready

    def send(self, msgs):
        for w, m in enumerate(msgs):
            self.conns[w].send(m)

    def close(self, abort=False):
        """Tell the workers to stop; they leave on their own (daemon processes, reaped by
        multiprocessing), so the walk does not wait for them.  After an error the
        workers may be blocked on each other: they are terminated."""
        for c in self.conns:
            try:
                c.send(("stop",))
                c.close()
            except (OSError, EOFError, BrokenPipeError):
                pass
        if abort:
            for pr in self.procs:
                if pr.is_alive():
                    pr.terminate()
        self.conns, self.procs = [], []


class _Walk:
    """Level-synchronous enumeration, serial while the levels are small, then sharded
    over worker processes (each owns the positions whose 128-bit fingerprint maps to
    it).  In the sharded part the parent never touches a position object: per level it
    merges the workers' (parent index, primitive, child count, child fingerprints),
    deduplicates and numbers the children with numpy against the sorted fingerprints
    of every position so far (new ones in first-occurrence order, so the numbering is
    the serial walk's), and tells each owner which of them it keeps -- the reference's
    owner-rank dedup (src/new_process.py:102-133, :145-162) with processes for ranks."""

    def __init__(self, module, gen_idx, workers, limit, budget_s):
        self.module, self.gen_idx, self.workers = module, list(gen_idx), workers
        self.gens = _generators(module, self.gen_idx)
        self.limit, self.budget_s = limit, budget_s
        self.index, self.positions = {}, []     # serial part
        self.prim, self.off, self.kids = [], [0], []
        self.sizes = []
        self.pool = None
        self.spec = _module_spec(module) if workers > 1 and _main_importable() else None
        self.n = 0                 # positions numbered so far
        self.G = self.GI = None    # sorted fingerprints of every position, and their indices
        self.members = 0           # orbit members of the positions the workers hold
        self.prim_parts, self.off_parts, self.kid_parts = [], [], []   # the parallel levels' CSR

    def _project(self, level_len, nxt_len, tl, t0):
        if not nxt_len:
            return 0
        growth = nxt_len / level_len
        projected = self.n + nxt_len * growth
        dt = time.perf_counter() - tl
        elapsed = time.perf_counter() - t0
        if projected > self.limit or (growth > 1 and elapsed + dt * growth * growth > self.budget_s):
            raise TooLarge(
                "plugin %s: after %d levels (sizes %s, %d positions, %.1f s) the next level is "
                "projected at ~%.3g positions (growth x%.2f per level): past the host-enumeration "
                "limits (%d positions, %.0f s); no device descriptor reproduces this plugin at these "
                "parameters" % (getattr(self.module, "__name__", self.module), len(self.sizes),
                                self.sizes + [nxt_len], self.n, elapsed, nxt_len * growth, growth, self.limit,
                                self.budget_s))
        return nxt_len * growth

    def _serial_level(self, level):
        nxt = []
        for pos in level:
            p, children = _expand_one(self.module, pos, self.gens)
            self.prim.append(p)
            for child in children:
                k = position_key(child)
                j = self.index.get(k)
                if j is None:
                    j = self.n
                    if j >= self.limit:
                        raise TooLarge("more than %d positions: too large for host enumeration (levels %s)"
                                       % (self.limit, self.sizes))
                    self.index[k] = j
                    self.positions.append(child)
                    self.n += 1
                    nxt.append(child)
                self.kids.append(j)
            self.off.append(len(self.kids))
        return nxt

    def _go_parallel(self, level):
        """Hand the current level to the workers' shards and the numbering to fingerprints."""
        self.pool.wait_ready()
        fps = [_fingerprint(p) for p in self.positions]
        G = np.frombuffer(b"".join(fps), dtype="V16")
        order = np.argsort(G, kind="stable")
        self.G, self.GI = G[order], order.astype(np.int64)
        self.G64, self.Glo = _halves(self.G)
        self.exact = bool(len(self.G64) > 1 and np.any(self.G64[1:] == self.G64[:-1]))
        self.nkids = len(self.kids)
        nw = self.pool.nw
        first = self.n - len(level)
        owned = [[] for _ in range(nw)]
        for f in fps[:first]:
            owned[_owner(f, nw)].append(f)
        shards = [[] for _ in range(nw)]
        for i, pos in enumerate(level):
            f = fps[first + i]
            owned[_owner(f, nw)].append(f)
            shards[_owner(f, nw)].append((f, pos))
        self.pool.send([("seed", b"".join(owned[w]), pickle.dumps(shards[w], protocol=4)) for w in range(nw)])
        self.pool.send([("run",)] * nw)

    def _lookup(self, F):
        """Indices of fingerprints every one of which the walk has numbered."""
        at = np.searchsorted(self.G, F) if self.exact else np.searchsorted(self.G64, _halves(F)[0])
        if len(F) and not (np.all(at < len(self.G)) and np.all(self.G[np.minimum(at, len(self.G) - 1)] == F)):
            raise RuntimeError("graph walk: a worker reported a position the walk never numbered")
        return self.GI[at]

    def _number_level(self, res):
        """Number one level from the workers' reports: its parents (numbered a level
        earlier) in index order, their children's fingerprints in that edge order; a child
        seen before gets its index, a new one the next index in first-occurrence order --
        the serial walk's numbering.  Returns the number of new positions.

        Fingerprints are compared by their first 8 bytes (one u64 sort per level) and
        checked on all 16; should two differ only in the last 8 (p ~ n^2 / 2^65), the
        level -- and every later one -- is numbered on the whole 16 bytes."""
        P = np.concatenate([np.frombuffer(r[1], dtype="V16") for r in res])
        prims = np.concatenate([np.frombuffer(r[2], dtype=np.uint8) for r in res])
        counts = np.concatenate([np.frombuffer(r[3], dtype=np.uint32) for r in res]).astype(np.int64)
        E = np.concatenate([np.frombuffer(r[4], dtype="V16") for r in res])
        idx = self._lookup(P)
        start = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        order = np.argsort(idx, kind="stable")
        if len(idx) and not np.array_equal(idx[order], np.arange(idx[order[0]], idx[order[0]] + len(idx))):
            raise RuntimeError("graph walk: the workers' parents are not one level of the walk")
        c = counts[order]
        tot = int(c.sum())
        csum = np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64)
        perm = np.repeat(start[order] - csum, c) + np.arange(tot, dtype=np.int64)
        E = E[perm]
        if len(prims) and int(prims.max()) > 4:
            raise ValueError("primitive() returned %r, not a src.utils code" % int(prims.max()))
        self.prim_parts.append(prims[order])
        self.off_parts.append(self.nkids + np.cumsum(c))
        self.nkids += tot
        if not tot:
            return 0
        hi, lo = _halves(E)
        fast = not self.exact
        if fast:
            o = np.argsort(hi)
            h = hi[o]
            flag = np.empty(tot, dtype=bool)
            flag[0] = True
            np.not_equal(h[1:], h[:-1], out=flag[1:])
            starts = np.flatnonzero(flag)
            uhi, first = h[starts], np.minimum.reduceat(o, starts)
            inv = np.empty(tot, dtype=np.int64)
            inv[o] = np.cumsum(flag) - 1
            ulo = lo[first]
            at = np.searchsorted(self.G64, uhi)
            found = np.zeros(len(uhi), dtype=bool)
            ok = at < len(self.G64)
            found[ok] = self.G64[at[ok]] == uhi[ok]
            fast = np.array_equal(lo, ulo[inv]) and np.array_equal(self.Glo[at[found]], ulo[found])
            uniq = E[first]
        if not fast:   # two fingerprints share their first 8 bytes: whole 16 from here on
            self.exact = True
            uniq, first, inv = np.unique(E, return_index=True, return_inverse=True)
            inv = inv.ravel()
            at = np.searchsorted(self.G, uniq)
            found = np.zeros(len(uniq), dtype=bool)
            ok = at < len(self.G)
            found[ok] = self.G[at[ok]] == uniq[ok]
        uidx = np.empty(len(uniq), dtype=np.int64)
        uidx[found] = self.GI[at[found]]
        new = np.flatnonzero(~found)
        new = new[np.argsort(first[new], kind="stable")]
        if self.n + len(new) > self.limit:
            raise TooLarge("more than %d positions: too large for host enumeration (levels %s)"
                           % (self.limit, self.sizes))
        uidx[new] = self.n + np.arange(len(new), dtype=np.int64)
        self.n += len(new)
        self.kid_parts.append(uidx[inv])
        ins = np.sort(new)   # positions of the new fingerprints in uniq (sorted by fingerprint)
        nh, nl = _halves(uniq[ins])
        self.G = np.insert(self.G, at[ins], uniq[ins])
        self.G64 = np.insert(self.G64, at[ins], nh)
        self.Glo = np.insert(self.Glo, at[ins], nl)
        self.GI = np.insert(self.GI, at[ins], uidx[ins])
        return len(new)

    def _parallel_levels(self, level_len, t0):
        """The workers run the levels on their own; number each from their reports."""
        nw = self.pool.nw
        trace = os.environ.get("GM_GRAPH_TRACE")
        while True:
            tl = time.perf_counter()
            res = [self.pool.recv(w, "level", "done") for w in range(nw)]
            kinds = {r[0] for r in res}
            if kinds == {"done"}:
                return
            if kinds != {"level"}:
                raise RuntimeError("graph walk: the workers disagree on the last level")
            t1 = time.perf_counter()
            if level_len:
                self.sizes.append(level_len)
            nxt_len = self._number_level(res)
            t2 = time.perf_counter()
            # the next level's position objects, now numbered
            pos = self.positions
            pos.extend([None] * (self.n - len(pos)))
            for w in range(nw):
                r = self.pool.recv(w, "adopted")
                F = np.frombuffer(r[1], dtype="V16")
                if len(F):
                    for i, p in zip(self._lookup(F).tolist(), pickle.loads(r[2])):
                        pos[i] = p
                self.members += r[3]
            if trace:
                import sys
                wt = [r[5] for r in res]
                print("[graph] level %d: %d parents, %d new | wait %.3f s (workers' expand max %.3f (w%d) min %.3f "
                      "(w%d); parents per worker %d-%d) number %.3f s adopted %.3f s"
                      % (len(self.sizes), level_len, nxt_len, t1 - tl, max(wt), wt.index(max(wt)), min(wt),
                         wt.index(min(wt)), min(len(r[2]) for r in res), max(len(r[2]) for r in res),
                         t2 - t1, time.perf_counter() - t2), file=sys.stderr)
            if level_len:
                self._project(level_len, nxt_len, tl, t0)
            level_len = nxt_len

    def _trace(self, what, t):
        if os.environ.get("GM_GRAPH_TRACE"):
            import sys
            print("[graph] %s %.3f s" % (what, time.perf_counter() - t), file=sys.stderr)

    def run(self, root):
        self.index[position_key(root)] = 0
        self.positions.append(root)
        self.n = 1
        level, level_len = [root], 1
        t0 = time.perf_counter()
        projected = 0
        spawned_at = None
        prestarted = False
        ok = False
        try:
            while level_len:
                tl = time.perf_counter()
                if self.spec is not None:
                    # workers are spawned once the graph is projected past PAR_START positions
                    # (tic-tac-toe never is: ADVICE r03); the parent keeps walking serially
                    # while they import, and hands over at the first level of PAR_MIN
                    # positions it meets with the workers ready (or 8 PAR_MIN, whatever)
                    # the fork server (one process) a level ahead of the workers, once the next
                    # level is projected past PAR_START / 8 positions at a growth of 4 or more
                    # per level (tic-tac-toe never is)
                    if not prestarted and 8 * projected >= PAR_START and projected >= 4 * level_len:
                        _prestart()
                        prestarted = True
                    if self.pool is None and (self.n + projected >= PAR_START or 2 * projected >= PAR_START
                                              or level_len >= 4 * PAR_MIN):
                        self.pool = _ShardPool(self.spec, self.workers, self.gen_idx)
                        spawned_at = len(self.sizes)
                        self._trace("spawn of %d workers at level %d (starts %s)" % (
                            self.workers, len(self.sizes) + 1, " ".join("%.3f" % x for x in self.pool.start_s)), tl)
                    # a pool started a level earlier is waited for (its workers start in ~50 ms,
                    # less than a serial level of PAR_MIN positions)
                    if self.pool is not None and level_len >= PAR_MIN and (
                            self.pool.poll_ready() or spawned_at < len(self.sizes) or level_len >= 8 * PAR_MIN):
                        tw = time.perf_counter()
                        self._go_parallel(level)
                        self._trace("workers ready (%s s after the spawn) and seeded" % " ".join(
                            "%.3f" % x for x in self.pool.ready_at), tw)
                        break
                self.sizes.append(level_len)
                level = self._serial_level(level)
                nxt_len = len(level)
                self._trace("serial level %d (%d positions)" % (len(self.sizes), level_len), tl)
                projected = self._project(level_len, nxt_len, tl, t0)
                level_len = nxt_len
            self.serial_positions = list(self.positions)
            if self.G is not None:   # the workers run the rest; the parent numbers it
                del level
                self._parallel_levels(level_len, t0)
            ok = True
        finally:
            if self.pool is not None:
                tc = time.perf_counter()
                self.pool.close(abort=not ok)
                self._trace("close", tc)
        self._trace("walk", t0)
        return (self.positions,
                np.concatenate([np.array(self.prim, dtype=np.uint8)] + self.prim_parts),
                np.concatenate([np.array(self.off, dtype=np.uint64)] + [a.astype(np.uint64) for a in self.off_parts]),
                np.concatenate([np.array(self.kids, dtype=np.uint32)] + [a.astype(np.uint32) for a in self.kid_parts]))


def enumerate_graph(module, root, limit=50_000_000, workers=None, budget_s=3600.0, symmetry=()):
    """Positions reachable from ``root`` (index 0) with primitive codes and CSR children.

    ``symmetry``: indices of ``symmetry_functions()`` that fix the root
    (symmetry_generators); the positions are then the orbit representatives.
    Raises TooLarge as soon as the projected next level would pass ``limit``
    positions or the walk's projected time would pass ``budget_s`` seconds."""
    workers = _default_workers() if workers is None else max(1, int(workers))
    root = canonical(root, _generators(module, list(symmetry)))
    return _Walk(module, symmetry, workers, limit, budget_s).run(root)


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
        workers = _default_workers() if workers is None else max(1, int(workers))
        walk = _Walk(module, self.symmetry, workers, 50_000_000, 3600.0)
        self.positions, self.prim, self.off, self.kids = walk.run(canonical(root, self.gens))
        self._index_map = None
        if self.gens:   # every orbit member counts (the workers counted theirs)
            self.n_positions = walk.members + sum(len(orbit(p, self.gens)) for p in walk.serial_positions)
        else:
            self.n_positions = len(self.positions)

    @property
    def _index(self):
        if self._index_map is None:   # built on first lookup, not on the solve path
            self._index_map = {position_key(p): i for i, p in enumerate(self.positions)}
        return self._index_map

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
