"""Worker side of the explicit-graph walk (gamesmanmpi_amd/graph.py), kept light.

The parallel walk spawns one process per host core; each imports only this module
(no numpy, no ctypes library -- the package's __init__ is lazy), rebuilds the plugin
from its file and owns the positions whose fingerprint maps to it.  The plugin calls
are the reference's expansion (GameState.expand, src/game_state.py:33-41: gen_moves +
do_move; primitive positions are not expanded, src/new_process.py:120-130); the
ownership mirrors its owner rank (src/game_state.py:23-31) and the one copy of each
child its owner keeps (lookup / distribute, src/new_process.py:102-162).
"""
import array
import hashlib
import importlib.util
import pickle
import time

UNDECIDED = 4


def _is_ndarray(x):
    t = type(x)
    return t.__name__ == "ndarray" and t.__module__ == "numpy"


def position_key(pos):
    """Hashable identity of a plugin position (numpy boards by dtype/shape/bytes)."""
    if _is_ndarray(pos):
        return ("ndarray", pos.dtype.str, pos.shape, pos.tobytes())
    return pos


def _order(pos):
    return pickle.dumps(position_key(pos), protocol=4)


def fingerprint(pos):
    """128-bit BLAKE2b digest of the position's identity: what the parallel walk
    deduplicates and numbers positions by (a collision needs ~2^64 positions; the walk
    is limited to 5e7).  str and int positions (the reference's plugins use both) hash
    a type tag and their text directly; anything else its pickled key."""
    t = type(pos)
    if t is str:
        b = b"s" + pos.encode("utf-8", "surrogatepass")
    elif t is int:
        b = b"i" + str(pos).encode()
    else:
        b = b"p" + _order(pos)
    return hashlib.blake2b(b, digest_size=16).digest()


def owner(fp, nw):
    return fp[0] % nw if nw <= 256 else int.from_bytes(fp[:4], "little") % nw


def generators(module, idx):
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


def expand_one(module, pos, gens=()):
    p = module.primitive(pos)
    if not (isinstance(p, int) or type(p).__module__ == "numpy") or not 0 <= int(p) <= 4:
        raise ValueError("primitive(%r) returned %r, not a src.utils code" % (pos, p))
    p = int(p)
    kids = [module.do_move(pos, m) for m in module.gen_moves(pos)] if p == UNDECIDED else []
    if gens:
        kids = [canonical(c, gens) for c in kids]
    return p, kids


def load_fresh(path, name="gm_graph_plugin"):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _exchange(peers, me, blobs):
    """All-to-all of one message per peer: a thread sends (a pipe holds ~64 KiB, so every
    worker sending before it receives would deadlock), this thread receives."""
    import threading
    nw = len(peers)

    def send():
        for k in range(1, nw):
            w = (me + k) % nw
            peers[w].send_bytes(blobs[w])
    th = threading.Thread(target=send, daemon=True)
    th.start()
    got = [b""] * nw
    for k in range(1, nw):
        w = (me - k) % nw
        got[w] = peers[w].recv_bytes()
    th.join()
    return got


def worker_main(conn, peers, me, path, attrs, gen_idx):
    """One shard of the parallel walk (a spawned process), the reference's rank
    (src/new_process.py:102-162) with pipes for MPI: it owns the positions whose
    fingerprint maps to it.  Seeded by the parent with the fingerprints it owns so far
    and its share of the current level, it then runs the levels on its own: expand its
    frontier, report (parent fingerprints, primitive codes, child counts, child
    fingerprints) to the parent, send each child object once to the child's owner
    (directly, one all-to-all per level over `peers`), keep the children it receives
    that it does not own yet as the next frontier (and send them to the parent, which
    keeps the position objects), and stop when every worker's frontier is empty.  The
    parent numbers the positions from the reports while the workers run the next
    level, off their critical path."""
    import traceback
    nw = len(peers)
    try:
        mod = load_fresh(path)
        for k, v in attrs.items():   # values the caller set on its module (board size, ...)
            setattr(mod, k, v)
        gens = generators(mod, list(gen_idx))
    except BaseException:
        conn.send(("error", traceback.format_exc()))
        return
    conn.send(("ready",))
    owned = set()
    frontier = []                       # (fingerprint, position) of the level to expand
    sent = set()      # fingerprints whose object this worker has already shipped
    try:
        while True:
            msg = conn.recv()
            if msg[0] == "seed":          # what it owns so far, and its share of the current level
                fp_b = msg[1]
                owned.update(fp_b[16 * j:16 * j + 16] for j in range(len(fp_b) // 16))
                frontier = pickle.loads(msg[2])
            elif msg[0] == "run":
                while True:
                    te = time.perf_counter()
                    prims = bytearray(len(frontier))
                    counts = array.array("I", bytes(4 * len(frontier)))
                    fps = []
                    out = [[] for _ in range(nw)]
                    for n, (_, pos) in enumerate(frontier):
                        p, kids = expand_one(mod, pos, gens)
                        prims[n] = p
                        counts[n] = len(kids)
                        for c in kids:
                            f = fingerprint(c)
                            fps.append(f)
                            if f not in sent:
                                sent.add(f)
                                out[owner(f, nw)].append((f, c))
                    conn.send(("level", b"".join(f for f, _ in frontier), bytes(prims), counts.tobytes(),
                               b"".join(fps), time.perf_counter() - te))
                    mine = out[me]
                    got = _exchange(peers, me, [pickle.dumps(o, protocol=4) if o else b"" for o in out])
                    frontier = []
                    for w in range(nw):   # fixed order: the frontier is the same on every run
                        for f, c in (mine if w == me else (pickle.loads(got[w]) if got[w] else ())):
                            if f not in owned:
                                owned.add(f)
                                frontier.append((f, c))
                    conn.send(("adopted", b"".join(f for f, _ in frontier),
                               pickle.dumps([c for _, c in frontier], protocol=4),
                               sum(len(orbit(c, gens)) for _, c in frontier) if gens else len(frontier)))
                    sizes = _exchange(peers, me, [b"%d" % len(frontier)] * nw)
                    if len(frontier) + sum(int(x) for w, x in enumerate(sizes) if w != me) == 0:
                        conn.send(("done",))
                        break
            elif msg[0] == "stop":
                return
    except BaseException:
        conn.send(("error", traceback.format_exc()))
