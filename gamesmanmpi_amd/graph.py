"""Any plugin on the device: explicit-graph solves (GM_GAME_GRAPH).

A plugin that no device descriptor reproduces (``games.identify`` returns None)
is still solved on the GPU: the host walks the plugin itself -- breadth-first
from the root with the reference's four functions (README.md:28-88; the same
expansion as GameState.expand, src/game_state.py:33-41, primitive positions not
expanded, src/new_process.py:120-130) -- numbers every distinct position, and
hands the graph to ``gm_solve_graph``, whose kernels run the retrograde.  Host
enumeration runs at Python speed; the device does the solving.  Positions must
be hashable, or numpy arrays (keyed by dtype, shape and bytes).
"""
import numpy as np

from . import _lib

UNDECIDED = 4


def position_key(pos):
    """Hashable identity of a plugin position (numpy boards by dtype/shape/bytes)."""
    if isinstance(pos, np.ndarray):
        return ("ndarray", pos.dtype.str, pos.shape, pos.tobytes())
    return pos


def enumerate_graph(module, root, limit=50_000_000):
    """Positions reachable from ``root`` (index 0) with primitive codes and CSR children."""
    index = {position_key(root): 0}
    positions = [root]
    prim = []
    off = [0]
    kids = []
    i = 0
    while i < len(positions):
        pos = positions[i]
        p = module.primitive(pos)
        if not isinstance(p, (int, np.integer)) or not 0 <= int(p) <= 4:
            raise ValueError("primitive(%r) returned %r, not a src.utils code" % (pos, p))
        prim.append(int(p))
        if p == UNDECIDED:
            for move in module.gen_moves(pos):
                child = module.do_move(pos, move)
                k = position_key(child)
                j = index.get(k)
                if j is None:
                    j = len(positions)
                    if j >= limit:
                        raise RuntimeError("more than %d positions: too large for host enumeration" % limit)
                    index[k] = j
                    positions.append(child)
                kids.append(j)
        off.append(len(kids))
        i += 1
    return positions, np.array(prim, dtype=np.uint8), np.array(off, dtype=np.uint64), np.array(kids, dtype=np.uint32)


class GraphCodec:
    """Keys of a graph solve are position indices; ``pos`` maps them back."""
    game_id = _lib.GAME_GRAPH
    params = ()
    name = "graph"

    def __init__(self, module, root):
        self.module = module
        self.positions, self.prim, self.off, self.kids = enumerate_graph(module, root)
        self._index = {position_key(p): i for i, p in enumerate(self.positions)}

    def key(self, pos):
        try:
            return self._index[position_key(pos)]
        except KeyError:
            raise ValueError("position not reachable from the root") from None

    def pos(self, key):
        return self.positions[int(key)]
