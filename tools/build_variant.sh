#!/bin/bash
# Development aid: build a libgmsolve variant with one source recompiled under extra
# flags:  tools/build_variant.sh NAME SOURCE -DFOO=1 ...  ->  _exp/libgm_NAME.so
# (load it with GM_LIB_PATH=_exp/libgm_NAME.so).  SOURCE e.g. dense_sub, sparse.
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
python -m gamesmanmpi_amd.build >/dev/null
mkdir -p _exp
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Igamesmanmpi_amd/csrc "$@" \
  -c gamesmanmpi_amd/csrc/$src.hip -o _exp/${src}_$name.o
objs=$(ls gamesmanmpi_amd/_build/*.o | grep -v "/$src.o")
hipcc -shared -fPIC --offload-arch=gfx950 $objs _exp/${src}_$name.o -o _exp/libgm_$name.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f _exp/libgm_$name.so.* _exp/${src}_$name.o
echo _exp/libgm_$name.so
