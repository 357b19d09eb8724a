import ctypes
import importlib.util
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)
if os.path.join(REPO, "oracle") not in sys.path:
    sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgmsolve.so on the device)")
    config.addinivalue_line("markers", "slow: long-running")


def load_plugin(rel, **attrs):
    """Load one of this repo's plugin modules as `game_module` (as the launcher does)."""
    import src.utils
    path = rel if os.path.isabs(rel) else os.path.join(REPO, rel)
    spec = importlib.util.spec_from_file_location("game_module", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for k, v in attrs.items():
        setattr(mod, k, v)
    src.utils.game_module = mod
    return mod


def golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return d["keys"], d["records"]


class Oracle:
    """ctypes view of oracle/_build/liboracle.so (test infrastructure)."""

    def __init__(self):
        path = os.path.join(REPO, "oracle", "_build", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.oracle_solve.restype = ctypes.c_int64
        L.oracle_solve.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, ctypes.c_uint64,
                                   P(P(ctypes.c_uint64)), P(P(ctypes.c_uint16))]
        L.oracle_initial.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_uint64)]
        L.oracle_expand.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, ctypes.c_uint64,
                                    P(ctypes.c_uint64), P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int64)]
        L.oracle_subtract_dense.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.oracle_subtract_dense_mt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.oracle_dense_digest.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, P(ctypes.c_uint64)]
        L.oracle_solve_layered.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, ctypes.c_uint64,
                                           ctypes.c_int, P(ctypes.c_uint64), P(ctypes.c_uint64),
                                           P(ctypes.c_uint16), P(ctypes.c_uint64), ctypes.c_int, P(ctypes.c_int)]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_free.argtypes = [ctypes.c_void_p]
        self.L = L

    def _params(self, params):
        params = list(params)
        return (ctypes.c_int32 * max(1, len(params)))(*params), len(params)

    def initial(self, game, params=()):
        p, n = self._params(params)
        r = ctypes.c_uint64()
        assert self.L.oracle_initial(game, p, n, ctypes.byref(r)) == 0
        return r.value

    def solve(self, game, params=(), root=None):
        p, n = self._params(params)
        if root is None:
            root = self.initial(game, params)
        kp, rp = ctypes.POINTER(ctypes.c_uint64)(), ctypes.POINTER(ctypes.c_uint16)()
        m = self.L.oracle_solve(game, p, n, root, ctypes.byref(kp), ctypes.byref(rp))
        if m < 0:
            raise RuntimeError(self.L.oracle_last_error().decode())
        keys = np.ctypeslib.as_array(kp, (m,)).copy() if m else np.zeros(0, np.uint64)
        recs = np.ctypeslib.as_array(rp, (m,)).copy() if m else np.zeros(0, np.uint16)
        self.L.oracle_free(kp)
        self.L.oracle_free(rp)
        return keys, recs

    def expand(self, game, params, key):
        p, n = self._params(params)
        kids = (ctypes.c_uint64 * 64)()
        nk, pr, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        assert self.L.oracle_expand(game, p, n, key, kids, ctypes.byref(nk), ctypes.byref(pr),
                                    ctypes.byref(t)) == 0
        return pr.value, sorted(kids[:nk.value]), t.value

    def subtract_dense(self, heaps):
        out = np.empty(1 << (4 * heaps), dtype=np.uint16)
        assert self.L.oracle_subtract_dense(heaps, out.ctypes.data) == 0
        return out

    def subtract_dense_mt(self, heaps, threads=0):
        out = np.empty(1 << (4 * heaps), dtype=np.uint16)
        assert self.L.oracle_subtract_dense_mt(heaps, out.ctypes.data, threads) == 0
        return out

    def dense_digest(self, recs, threads=0):
        """gm_digest of a dense table (key = index), computed by the oracle library."""
        d = ctypes.c_uint64()
        recs = np.ascontiguousarray(recs, dtype=np.uint16)
        assert self.L.oracle_dense_digest(recs.ctypes.data, ctypes.c_uint64(len(recs)), threads,
                                          ctypes.byref(d)) == 0
        return d.value

    def solve_layered(self, game, params=(), root=None, threads=0):
        """Sorted-layer OpenMP solver: (positions, digest, root record, per-tier counts)."""
        p, n = self._params(params)
        if root is None:
            root = self.initial(game, params)
        npos, dg, rr, nt = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint16(), ctypes.c_int()
        tiers = (ctypes.c_uint64 * 4096)()
        if self.L.oracle_solve_layered(game, p, n, ctypes.c_uint64(root), threads, ctypes.byref(npos),
                                       ctypes.byref(dg), ctypes.byref(rr), tiers, 4096, ctypes.byref(nt)) != 0:
            raise RuntimeError(self.L.oracle_last_error().decode())
        return npos.value, dg.value, rr.value, [int(x) for x in tiers[:nt.value]]


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


def digest(keys, recs):
    """Same order-independent digest as gm_digest (include/gmsolve.h)."""
    k = keys.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = k * np.uint64(0x9E3779B97F4A7C15) + recs.astype(np.uint64)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xff51afd7ed558ccd)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xc4ceb9fe1a85ec53)
        x ^= x >> np.uint64(33)
        return int(x.sum(dtype=np.uint64))
