"""Build libgmsolve.so (HIP, gfx950) in-tree with hipcc.

    python -m gamesmanmpi_amd.build [--jobs N] [--verbose]

Objects go to gamesmanmpi_amd/_build/, the library to gamesmanmpi_amd/libgmsolve.so
(git-ignored, but it travels to the GPU box with the gpurun snapshot).
"""
import argparse
import concurrent.futures
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libgmsolve.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("GM_OFFLOAD_ARCH", "gfx950")

SOURCES = ["gm_api.hip", "dense_sub.hip", "dense_box.hip", "dist_box.hip", "small_dense.hip", "sparse.hip", "dist_sub.hip",
           "dist_sparse.hip",
           "graph.hip"]
HEADERS = ["gm_common.hpp", "box_common.hpp", "games.hpp", "gm_internal.hpp", "sparse_common.hpp", "sparse_tables.hpp"]

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result",
            "-I" + os.path.join(REPO, "include"), "-I" + CSRC]


def hipcc():
    exe = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(exe):
        raise RuntimeError("hipcc not found (ROCm %s)" % ROCM)
    return exe


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, verbose):
    out = os.path.join(OBJ, os.path.splitext(os.path.basename(src))[0] + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "gmsolve.h")]
    if not _stale(out, deps):
        return out
    cmd = [hipcc(), *CXXFLAGS, "-c", src, "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError("hipcc failed on %s:\n%s%s" % (src, r.stdout, r.stderr))
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    return out


def build(jobs=None, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    jobs = jobs or min(8, len(srcs))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    if _stale(LIB, objs):
        cmd = [hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH, *objs, "-o", LIB,
               "-L" + os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib")]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("link failed:\n%s%s" % (r.stdout, r.stderr))
    # the device link leaves per-arch temporaries next to the library
    import glob
    for tmp in glob.glob(LIB + ".*-*"):
        os.remove(tmp)
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.verbose))


if __name__ == "__main__":
    main()
