"""gamesmanmpi_amd -- MI355X-native strong solver behind GamesmanMPI's plugin API.

The solve path is libgmsolve.so (hand-written HIP for gfx950, C ABI in
include/gmsolve.h); this package is the Python host above it.  Its names load on
first use, so a process that imports one submodule (the graph walk's workers import
gamesmanmpi_amd.walk_worker) does not import numpy or load the library.
"""
import importlib

_NAMES = {"GMError": "._lib", "lib": "._lib", "Context": ".solver", "NoDescriptor": ".solver",
          "Solver": ".solver", "split_record": ".solver"}

__all__ = ["Solver", "Context", "GMError", "NoDescriptor", "split_record", "games", "lib"]


def __getattr__(name):
    if name in _NAMES:
        return getattr(importlib.import_module(_NAMES[name], __name__), name)
    if name == "games":
        return importlib.import_module(".games", __name__)
    raise AttributeError("module %r has no attribute %r" % (__name__, name))
