"""Time of starting the graph walk's spawned worker pool, first and second time in one
process (development aid for gamesmanmpi_amd/graph.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import multiprocessing as mp
    from gamesmanmpi_amd import graph
    ctx = mp.get_context("spawn")
    for rep in range(3):
        t0 = time.perf_counter()
        a, b = ctx.Pipe()
        t1 = time.perf_counter()
        ps = []
        for w in range(16):
            ts = time.perf_counter()
            p = ctx.Process(target=graph._noop_worker if hasattr(graph, "_noop_worker") else time.sleep, args=(0.2,),
                            daemon=True)
            p.start()
            ps.append(time.perf_counter() - ts)
        t2 = time.perf_counter()
        for p in []:
            p.join()
        print("rep %d: pipe %.4f s, 16 starts %.3f s (each %s)" % (rep, t1 - t0, t2 - t1,
                                                                  " ".join("%.3f" % x for x in ps)), flush=True)
        time.sleep(0.5)


if __name__ == "__main__":
    main()
