"""Code fingerprints of game plugins: which plugin files a device descriptor is KNOWN to reproduce.

A plugin (``initial_position / gen_moves / do_move / primitive``, reference
README.md:28-88) is bound to a device descriptor (games.identify) only when that
binding is certain -- sampling a few hundred positions cannot tell a plugin from
one that differs only in deep or rare positions.  Certainty comes from one of:

* its code is one of the plugin files the descriptors were written from and tested
  against: the reference's ``test_games/{four_to_one,mttt,tic_tac_toe_np,
  toot_and_otto_bitstring,othello_bit_new}.py`` and this repo's ``test_games/*.py``.
  The fingerprint is a SHA-256 over the bytecode of the three rule functions
  (``gen_moves``, ``do_move``, ``primitive``) and of
  everything they reach -- module functions they call (transitively), closures
  (the ``src.utils`` encode/decode decorators), default arguments, and the values of
  the module globals they read (``BLANK``, ``MAX_TAKE``, ...).  Board dimensions
  and heap counts (``length``, ``height``, ``area``, ``HEAPS``) are left out: they
  are the descriptor's parameters, read from the module by the codec;
* or an exhaustive cross-check of every reachable position (games.identify).

``initial_position`` does not enter it either: it only names the root, which the solver
is handed explicitly and checks on its own (the codec must encode it, and the plugin and
the descriptor must agree on positions sampled below it).  The launcher's ``--custom FILE
--init_pos NAME`` replaces that function, as the reference's does (solver_launcher.py:106-111),
and a plugin solved from another root keeps its binding.

Docstrings and line numbers do not enter the hash; any change of code or of a
constant does.  Bytecode is interpreter-specific, so the stored fingerprints carry
the Python version they were made with and only match under it.

    python -m gamesmanmpi_amd.fingerprint --write    # regenerate plugin_fingerprints.json
"""
import builtins
import hashlib
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
STORE = os.path.join(HERE, "plugin_fingerprints.json")
PARAM_NAMES = frozenset({"length", "height", "area", "HEAPS"})
RULES = ("gen_moves", "do_move", "primitive")
_SIMPLE = (int, float, complex, str, bytes, bool, type(None))


def _simple_repr(v):
    """A stable repr for constants (None when v is not plain data)."""
    if isinstance(v, _SIMPLE):
        return repr(v)
    if isinstance(v, (tuple, list)):
        parts = [_simple_repr(x) for x in v]
        return None if None in parts else type(v).__name__ + "(" + ",".join(parts) + ")"
    if isinstance(v, (set, frozenset)):
        parts = sorted(_simple_repr(x) or "?" for x in v)
        return None if "?" in parts else "set(" + ",".join(parts) + ")"
    if isinstance(v, dict):
        items = sorted((_simple_repr(k) or "?", _simple_repr(x) or "?") for k, x in v.items())
        return None if any("?" in kv for kv in items) else "dict(" + ",".join("%s:%s" % kv for kv in items) + ")"
    return None


class _Hasher:
    def __init__(self):
        self.h = hashlib.sha256()
        self.seen = set()

    def put(self, *parts):
        for p in parts:
            self.h.update(p if isinstance(p, bytes) else str(p).encode())
            self.h.update(b"\0")

    def code(self, co, is_function):
        self.put("code", co.co_argcount, co.co_kwonlyargcount, co.co_flags, co.co_code, repr(co.co_names))
        consts = co.co_consts
        if is_function and consts and isinstance(consts[0], str):
            consts = consts[1:]   # the docstring
        for c in consts:
            if isinstance(c, types.CodeType):
                self.code(c, False)
            else:
                self.put("const", _simple_repr(c) or type(c).__name__)

    def names(self, co):
        out = set(co.co_names)
        for c in co.co_consts:
            if isinstance(c, types.CodeType):
                out |= self.names(c)
        return out

    def value(self, name, v):
        if name in PARAM_NAMES:
            self.put("param", name)
        elif isinstance(v, (types.FunctionType, types.MethodType)):
            self.put("fn", name)
            self.function(getattr(v, "__func__", v))
        elif _simple_repr(v) is not None:
            self.put("value", name, _simple_repr(v))
        elif isinstance(v, types.ModuleType):
            self.put("module", name, v.__name__)
            if v.__name__ == "src.utils":   # the result codes the plugins return
                self.put("codes", _simple_repr(tuple(getattr(v, c, None) for c in
                                                     ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED"))))
        elif isinstance(v, type):
            self.put("type", name, v.__module__, v.__qualname__)
        elif isinstance(v, types.BuiltinFunctionType):
            self.put("builtin", name, getattr(v, "__module__", ""), v.__qualname__)
        else:
            self.put("object", name, type(v).__module__, type(v).__qualname__)

    def function(self, f):
        if id(f) in self.seen:
            self.put("again", f.__qualname__)
            return
        self.seen.add(id(f))
        co = f.__code__
        self.code(co, True)
        self.put("defaults", _simple_repr(f.__defaults__ or ()))
        for cell, var in zip(f.__closure__ or (), co.co_freevars):
            try:
                self.value(var, cell.cell_contents)
            except ValueError:   # empty cell
                self.put("cell", var)
        g = f.__globals__
        for name in sorted(self.names(co)):
            if name in g:
                self.value(name, g[name])
            elif hasattr(builtins, name):
                self.put("builtin", name)
            else:
                self.put("attr", name)   # an attribute name (obj.name): in co_names, not a global


def fingerprint(module):
    """SHA-256 hex digest of the plugin's game code (module docstring for the rules)."""
    h = _Hasher()
    h.put("python", "%d.%d" % sys.version_info[:2])
    for name in RULES:
        f = getattr(module, name, None)
        h.put("api", name)
        if isinstance(f, (types.FunctionType, types.MethodType)):
            h.function(getattr(f, "__func__", f))
        else:
            h.put("missing" if f is None else type(f).__qualname__)
    return h.h.hexdigest()


_known = None


def known():
    """{fingerprint: {"codec": name, "source": path}} of the stored plugin files.

    Fingerprints hash bytecode, so they only match under the Python version the store was
    made with; under another one this warns (once) that no known plugin file will be
    recognised -- plugins then bind only by the exhaustive check, and large ones go to
    the graph engine -- instead of losing the device path silently."""
    global _known
    if _known is None:
        try:
            with open(STORE) as f:
                data = json.load(f)
            _known = data["fingerprints"]
            made = data.get("python")
            here = "%d.%d" % sys.version_info[:2]
            if made and made != here:
                import warnings
                warnings.warn("gamesmanmpi_amd: plugin fingerprints were made under Python %s, this is %s: "
                              "no plugin file will be recognised by its code (run `python -m "
                              "gamesmanmpi_amd.fingerprint --write` under this interpreter)" % (made, here),
                              RuntimeWarning, stacklevel=2)
        except (OSError, ValueError, KeyError):
            _known = {}
    return _known


# plugin file -> codec name it must bind to (the reference's own files, and this repo's rewrites)
SOURCES = [
    ("test_games/four_to_one.py", "four_to_one"),
    ("test_games/mttt.py", "mttt"),
    ("test_games/tic_tac_toe_np.py", "tic_tac_toe_np"),
    ("test_games/toot_and_otto_bitstring.py", "toot_and_otto"),
    ("test_games/othello_bit_new.py", "othello"),
    ("test_games/subtraction.py", "subtraction"),
]
REFERENCE = "/root/reference"


def _load(path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("fp_plugin", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _stub_reference_imports():
    """Importing the reference's plugin files needs mpi4py (tic_tac_toe_np.py:2, unused)
    and the third-party bitstring (not installed): stand-ins that only let the module
    load -- the fingerprint reads code, it runs nothing."""
    if "mpi4py" not in sys.modules:
        m = types.ModuleType("mpi4py")
        m.MPI = types.ModuleType("mpi4py.MPI")
        sys.modules["mpi4py"] = m
        sys.modules["mpi4py.MPI"] = m.MPI
    if "bitstring" not in sys.modules:
        b = types.ModuleType("bitstring")

        class BitArray:
            pass
        BitArray.__module__ = "bitstring"
        b.BitArray = BitArray
        sys.modules["bitstring"] = b


def generate():
    repo = os.path.dirname(HERE)
    sys.path.insert(0, repo)
    import src.utils  # noqa: F401  (plugins import this repo's src.utils, as under the launcher)
    out = {}
    for rel, codec in SOURCES:
        out[fingerprint(_load(os.path.join(repo, rel)))] = {"codec": codec, "source": rel}
    if os.path.isdir(REFERENCE):
        _stub_reference_imports()
        for rel, codec in SOURCES:
            path = os.path.join(REFERENCE, rel)
            if os.path.exists(path):
                out[fingerprint(_load(path))] = {"codec": codec, "source": "reference " + rel}
    return out


if __name__ == "__main__":
    if "--write" in sys.argv:
        fps = generate()
        with open(STORE, "w") as f:
            json.dump({"python": "%d.%d" % sys.version_info[:2],
                       "made_by": "python -m gamesmanmpi_amd.fingerprint --write",
                       "fingerprints": fps}, f, indent=1, sort_keys=True)
            f.write("\n")
        print("%d fingerprints -> %s" % (len(fps), STORE))
    else:
        for k, v in sorted(generate().items(), key=lambda kv: kv[1]["source"]):
            print(k, v["codec"], v["source"])
