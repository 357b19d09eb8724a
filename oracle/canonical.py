"""CPU oracle (pure Python): canonical strong solve over any GamesmanMPI plugin module.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``gamesmanmpi_amd``, ``solver_launcher.py``,
``solve_local.py``) never calls it.

Semantics (the parity contract):

* the position set is the closure of the root under ``do_move(p, m)`` for
  ``m in gen_moves(p)``; primitive positions are not expanded
  (reference ``src/new_process.py:102-133``: ``lookup`` returns before ``distribute``);
* a primitive position has value ``primitive(p)`` and remoteness 0
  (``PRIMITIVE_REMOTENESS``, ``src/utils.py:7``; stored at ``src/new_process.py:122``);
* otherwise the best child is chosen as ``GameState.compare_gamestates`` does
  (``src/game_state.py:105-125``): a LOSS child with the smallest remoteness, else
  a TIE child with the smallest remoteness, else (all WIN) the WIN child with the
  largest remoteness; the value is ``Process._res_red`` of that child
  (``src/new_process.py:189-198``: TIE -> TIE, LOSS -> WIN, else LOSS) and the
  remoteness is the child's + 1 (``src/new_process.py:250``).

DRAW primitives are rejected: the reference's fold makes DRAW and TIE children
order-dependent (``src/utils.py:90-96`` ``<=`` tie rule) and no config produces
DRAW.  A non-primitive position without moves is rejected (the reference hangs
there: ``_counter`` stays 0, ``src/new_process.py:135-162``).
"""
import numpy as np

WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4


class OracleError(RuntimeError):
    pass


def default_key(pos):
    """Hashable identity of a position (numpy boards by their bytes)."""
    if isinstance(pos, np.ndarray):
        return (pos.shape, pos.dtype.str, pos.tobytes())
    return pos


def fold(children):
    """Appendix A reduction of a list of child ``(value, remoteness)`` pairs."""
    best_loss = None
    best_tie = None
    worst_win = None
    for v, r in children:
        if v == LOSS:
            best_loss = r if best_loss is None else min(best_loss, r)
        elif v == TIE:
            best_tie = r if best_tie is None else min(best_tie, r)
        elif v == WIN:
            worst_win = r if worst_win is None else max(worst_win, r)
        else:
            raise OracleError("child value %r is not WIN/LOSS/TIE" % (v,))
    if best_loss is not None:
        return WIN, best_loss + 1
    if best_tie is not None:
        return TIE, best_tie + 1
    if worst_win is None:
        raise OracleError("non-primitive position without children")
    return LOSS, worst_win + 1


def solve(module, root=None, key=default_key, limit=None):
    """Strong-solve ``module`` from ``root`` (default ``initial_position()``).

    Returns ``(table, positions)``: ``table[key(p)] = (value, remoteness)`` and
    ``positions[key(p)] = p`` for every reachable position ``p``.
    """
    if root is None:
        root = module.initial_position()
    table = {}
    positions = {}
    children_of = {}
    rk = key(root)
    positions[rk] = root
    stack = [rk]
    gray = set()   # expanded, waiting for children: the current DFS path
    while stack:
        k = stack[-1]
        if k in table:
            stack.pop()
            continue
        pos = positions[k]
        kids = children_of.get(k)
        if kids is None:
            prim = module.primitive(pos)
            if prim == DRAW:
                raise OracleError("DRAW primitive is not supported")
            if prim in (WIN, LOSS, TIE):
                table[k] = (prim, 0)
                stack.pop()
                continue
            if prim != UNDECIDED:
                raise OracleError("primitive() returned %r" % (prim,))
            kids = []
            for m in module.gen_moves(pos):
                child = module.do_move(pos, m)
                ck = key(child)
                positions.setdefault(ck, child)
                kids.append(ck)
            if not kids:
                raise OracleError("non-primitive position without moves: %r" % (pos,))
            children_of[k] = kids
            gray.add(k)
            if limit is not None and len(positions) > limit:
                raise OracleError("position limit exceeded")
        pending = [c for c in kids if c not in table]
        if not pending:
            table[k] = fold(table[c] for c in kids)
            del children_of[k]
            gray.discard(k)
            stack.pop()
            continue
        for c in pending:
            if c in gray:
                raise OracleError("cycle through %r" % (positions[c],))
            stack.append(c)
    return table, positions


def root_line(value, remoteness):
    """The reference's root line ``"<V> in <R> moves"`` (``src/new_process.py:47-52``)."""
    return "%s in %d moves" % (("WIN", "LOSS", "TIE", "DRAW")[value], remoteness)
