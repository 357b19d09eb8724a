"""Host enumeration time of the explicit-graph path (gamesmanmpi_amd/graph.py) on a plugin
forced off its device descriptor: Toot-and-Otto 4x3 (200,127 positions) by default.

    python tools/graph_enum_time.py [workers ...]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from conftest import load_plugin
    from gamesmanmpi_amd.graph import _default_workers, enumerate_graph
    mod = load_plugin("test_games/toot_and_otto_bitstring.py", length=4, height=3)
    for w in [int(x) for x in sys.argv[1:]] or [1, _default_workers()]:
        t = time.perf_counter()
        pos, prim, off, kids = enumerate_graph(mod, mod.initial_position(), workers=w)
        print("Toot 4x3 graph enumeration: %d positions, %d edges, %d workers: %.2f s"
              % (len(pos), len(kids), w, time.perf_counter() - t), flush=True)


if __name__ == "__main__":
    main()
