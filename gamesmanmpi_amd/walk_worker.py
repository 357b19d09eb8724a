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
import os
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


class _Sender:
    """Sends from a thread, in order: the worker's own thread never blocks on a full pipe
    (a pipe holds ~64 KiB; two workers blocked on sends to each other would deadlock)."""

    def __init__(self):
        import queue
        import threading
        self.q = queue.Queue()
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            conn, data = item
            if isinstance(data, bytes):
                conn.send_bytes(data)
            else:
                conn.send(data)

    def put(self, conn, data):
        self.q.put((conn, data))

    def close(self):
        self.q.put(None)
        self.th.join()


class _Level:
    """What a worker reports to the parent for one level it expanded."""

    def __init__(self):
        self.pfps, self.kfps = [], []
        self.prims = bytearray()
        self.counts = array.array("I")
        self.t = 0.0


CHUNK = 64    # positions expanded between two looks at the incoming pipes (GM_GRAPH_CHUNK)


HANDSHAKE_S = 5.0   # a connection's HMAC challenge and peer number must arrive within this


def _mesh(me, nw, tag, key, timeout_s=120.0):
    """Pipes to every other worker: worker w listens on an abstract unix socket named by
    the walk's tag and w, connects to every lower-numbered worker's and accepts every
    higher-numbered one's.  Abstract socket names are visible to every process of the
    network namespace (/proc/net/unix) and the peers exchange pickles, so each connection
    is authenticated with the walk's random key (multiprocessing's HMAC challenge); one
    that fails it is dropped.  The workers build the mesh themselves so the parent never holds
    the n(n-1) descriptors (growing a threaded process's descriptor table waits for an RCU
    grace period, ~0.1 s a doubling on a busy host).  Everything is bounded by timeout_s
    (ADVICE r04): the accept loop polls, and a connection's challenge and its first message
    must arrive within HANDSHAKE_S (a socket receive timeout, cleared once it is a peer),
    so a local process that connects and never answers, or a peer that died before
    connecting, ends the mesh with TimeoutError -- worker_main reports it to the parent."""
    import socket
    import struct
    from multiprocessing import AuthenticationError
    from multiprocessing.connection import Connection, answer_challenge, deliver_challenge
    name = "\0" + tag + "-%d"
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(name % me)
    srv.listen(max(1, nw))
    srv.settimeout(0.25)
    peers = [None] * nw
    deadline = time.time() + timeout_s

    def rcvtimeo(c, secs):   # SO_RCVTIMEO on the connection's descriptor (0 = none)
        so = socket.socket(fileno=c.fileno())
        try:
            so.setsockopt(socket.SOL_SOCKET, socket.SO_RCVTIMEO, struct.pack("ll", int(secs), 0))
        finally:
            so.detach()

    try:
        for p in range(me):
            # connecting side: a raw socket with a connect timeout, then the
            # challenge exchange under SO_RCVTIMEO, so a lower-numbered peer that accepted but
            # never answers ends the mesh with TimeoutError too
            while True:
                so = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                try:
                    so.settimeout(max(0.05, deadline - time.time()))
                    so.connect(name % p)
                    break
                except (FileNotFoundError, ConnectionRefusedError, socket.timeout):
                    so.close()
                    if time.time() > deadline:
                        raise TimeoutError("walk worker %d: peer %d did not accept within %.0f s" % (me, p, timeout_s))
                    time.sleep(0.002)
            so.settimeout(None)
            c = Connection(so.detach())
            try:
                rcvtimeo(c, max(1.0, min(HANDSHAKE_S, deadline - time.time())))
                answer_challenge(c, key)
                deliver_challenge(c, key)
                c.send_bytes(b"%d" % me)
                rcvtimeo(c, 0)
            except (EOFError, OSError) as e:
                c.close()
                raise TimeoutError("walk worker %d: handshake with peer %d failed or timed out (%s)" % (me, p, e))
            peers[p] = c
        left = nw - 1 - me
        while left:
            if time.time() > deadline:
                raise TimeoutError("walk worker %d: %d higher-numbered peers did not connect within %.0f s"
                                   % (me, left, timeout_s))
            try:
                s, _ = srv.accept()
            except socket.timeout:
                continue
            s.settimeout(None)
            c = Connection(s.detach())
            try:
                rcvtimeo(c, max(1.0, min(HANDSHAKE_S, deadline - time.time())))
                deliver_challenge(c, key)
                answer_challenge(c, key)
                w = int(c.recv_bytes())
                if not (me < w < nw) or peers[w] is not None:
                    raise ValueError("bad peer number %d" % w)
                rcvtimeo(c, 0)
            except (AuthenticationError, EOFError, OSError, ValueError):
                c.close()
                continue
            peers[w] = c
            left -= 1
    finally:
        srv.close()
    return peers


def worker_main(conn, me, nw, tag, key, path, attrs, gen_idx):
    """One shard of the parallel walk (a spawned process), the reference's rank
    (src/new_process.py:102-162) with pipes for MPI: it owns the positions whose
    fingerprint maps to it.  Seeded by the parent with the fingerprints it owns so far
    and its share of the current level, it then runs on its own: it expands its
    frontier a chunk at a time, sends each child object once to the child's owner
    (directly, tagged with the level), keeps the children it receives that it does not
    own yet as the next level's frontier, and reports every level to the parent
    (parent fingerprints, primitive codes, child counts, child fingerprints; then the
    positions it took for the next level).  Levels overlap: a worker expands the part of
    level L + 1 it already has while a slower worker finishes level L; a level-L child
    is taken (or found known) only once every worker's level L - 1 children are in, so a
    position's level is its breadth-first depth and the parent's numbering, a level
    behind, is the serial walk's.  It stops when every worker's frontier of one level is
    empty."""
    import traceback
    from multiprocessing.connection import wait
    from collections import defaultdict
    try:
        peers = _mesh(me, nw, tag, key)
        mod = load_fresh(path)
        for k, v in attrs.items():   # values the caller set on its module (board size, ...)
            setattr(mod, k, v)
        gens = generators(mod, list(gen_idx))
    except BaseException:
        conn.send(("error", traceback.format_exc()))
        return
    conn.send(("ready", time.time()))
    chunk_n = int(os.environ.get("GM_GRAPH_CHUNK", CHUNK))
    try:
        msg = conn.recv()
        if msg[0] != "seed":
            return
        fp_b = msg[1]
        owned = set(fp_b[16 * j:16 * j + 16] for j in range(len(fp_b) // 16))
        frontier = {0: pickle.loads(msg[2])}
        if conn.recv()[0] != "run":
            return
        out = _Sender()      # to the peers, in order
        up = _Sender()       # to the parent (which reads the workers in turn)
        others = [peers[w] for w in range(nw) if w != me]
        sent = set()         # fingerprints whose object this worker shipped in this level (kept
                             # per level: a child of a tiered game is one level down only, and the
                             # owner deduplicates anyway; a walk-long set would grow with the edges)
        acc = 0              # level-acc children are applied on arrival; frontier[acc + 1] is filling
        ends = defaultdict(int)          # level -> workers done expanding it
        busy = defaultdict(bool)         # level -> some worker's frontier was non-empty
        held = defaultdict(list)         # level -> children that arrived early
        lvl, i, rep = 0, 0, _Level()     # expansion cursor and its report
        state = {"done": False}

        def apply(tag, items):
            nxt = frontier.setdefault(tag + 1, [])
            for f, c in items:
                if f not in owned:
                    owned.add(f)
                    nxt.append((f, c))

        def take(tag, items):
            if tag == acc:
                apply(tag, items)
            else:
                held[tag].append(items)

        def advance():
            nonlocal acc
            while ends[acc] == nw and not state["done"]:
                nxt = frontier.setdefault(acc + 1, [])   # complete: every level-acc child is in
                up.put(conn, ("adopted", b"".join(f for f, _ in nxt), pickle.dumps([c for _, c in nxt], protocol=4),
                              sum(len(orbit(c, gens)) for _, c in nxt) if gens else len(nxt)))
                if not busy[acc]:
                    state["done"] = True
                    return
                acc += 1
                for items in held.pop(acc, []):
                    apply(acc, items)

        def on_message(c):
            if c is conn:
                m = conn.recv()
                if m[0] == "stop":
                    raise SystemExit
                return
            kind, tag, payload = pickle.loads(c.recv_bytes())
            if kind == "kids":
                take(tag, payload)
            else:   # "end": the sender expanded all of its level `tag`
                ends[tag] += 1
                busy[tag] = busy[tag] or payload
                advance()

        while not state["done"]:
            F = frontier.setdefault(lvl, [])
            if i < len(F):
                te = time.perf_counter()
                chunk = F[i:i + chunk_n]
                i += len(chunk)
                dest = [[] for _ in range(nw)]
                for f0, pos in chunk:
                    p, kids = expand_one(mod, pos, gens)
                    rep.pfps.append(f0)
                    rep.prims.append(p)
                    rep.counts.append(len(kids))
                    for c in kids:
                        f = fingerprint(c)
                        rep.kfps.append(f)
                        if f not in sent:
                            sent.add(f)
                            dest[owner(f, nw)].append((f, c))
                for w in range(nw):
                    if w == me:
                        if dest[w]:
                            take(lvl, dest[w])
                    elif dest[w]:
                        out.put(peers[w], pickle.dumps(("kids", lvl, dest[w]), protocol=4))
                rep.t += time.perf_counter() - te
                for c in wait(others + [conn], timeout=0):
                    on_message(c)
            elif lvl <= acc:   # level lvl is complete and expanded
                up.put(conn, ("level", b"".join(rep.pfps), bytes(rep.prims), rep.counts.tobytes(),
                              b"".join(rep.kfps), rep.t))
                end = pickle.dumps(("end", lvl, len(F) > 0), protocol=4)
                for c in others:
                    out.put(c, end)
                ends[lvl] += 1
                busy[lvl] = busy[lvl] or len(F) > 0
                del frontier[lvl]
                lvl, i, rep = lvl + 1, 0, _Level()
                sent.clear()
                advance()
            else:              # wait for the rest of this level's frontier
                for c in wait(others + [conn]):
                    on_message(c)
        out.close()
        up.put(conn, ("done",))
        up.close()
        while conn.recv()[0] != "stop":
            pass
    except SystemExit:
        return
    except BaseException:
        try:
            conn.send(("error", traceback.format_exc()))
        except Exception:
            pass
