"""DescToot::child_at (csrc/games.hpp), which the sparse engine's MLP kernels use to make a
parent's children in registers, against visit(), which every other kernel and the host
twin use: the same children in the same order for every position of Toot 4x3 and 4x4,
with and without the mirror reduction (tools/child_at_check.cpp, compiled here)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = CXX if os.path.exists(CXX) else shutil.which("clang++")
    if not cxx:
        pytest.skip("no clang++ to build the host check")
    exe = str(tmp_path_factory.mktemp("child_at") / "child_at_check")
    subprocess.run([cxx, "-O2", "-std=c++17", "-include", "type_traits", "-I",
                    os.path.join(REPO, "gamesmanmpi_amd", "csrc"), os.path.join(REPO, "tools", "child_at_check.cpp"),
                    "-o", exe], check=True, timeout=300)
    return exe


@pytest.mark.parametrize("dims", [(4, 3), (4, 4), (3, 3)])
def test_child_at_equals_visit(checker, dims):
    r = subprocess.run([checker, *map(str, dims)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
