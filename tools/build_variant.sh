#!/bin/bash
# Development aid: build a libgmsolve variant with dense_sub.hip compiled under extra
# flags:  tools/build_variant.sh NAME -DFOO=1 ...  ->  _exp/libgm_NAME.so (GM_LIB_PATH=...)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
python -m gamesmanmpi_amd.build >/dev/null
mkdir -p _exp
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Igamesmanmpi_amd/csrc "$@" \
  -c gamesmanmpi_amd/csrc/dense_sub.hip -o _exp/dense_sub_$name.o
objs=$(ls gamesmanmpi_amd/_build/*.o | grep -v dense_sub.o)
hipcc -shared -fPIC --offload-arch=gfx950 $objs _exp/dense_sub_$name.o -o _exp/libgm_$name.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f _exp/libgm_$name.so.*
echo _exp/libgm_$name.so
