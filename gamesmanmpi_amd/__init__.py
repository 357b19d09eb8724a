"""gamesmanmpi_amd -- MI355X-native strong solver behind GamesmanMPI's plugin API.

The solve path is libgmsolve.so (hand-written HIP for gfx950, C ABI in
include/gmsolve.h); this package is the Python host above it.
"""
from ._lib import GMError, lib  # noqa: F401
from .solver import Context, NoDescriptor, Solver, split_record  # noqa: F401
from . import games  # noqa: F401

__all__ = ["Solver", "Context", "GMError", "NoDescriptor", "split_record", "games", "lib"]
