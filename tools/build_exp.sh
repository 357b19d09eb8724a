#!/bin/bash
# Development aid: build libgmsolve variants with dense_sub.hip compiled under
# -DGM_EXP=<n> into _exp/libgm_exp<n>.so (load with GM_LIB_PATH=...).
set -e
cd "$(dirname "$0")/.."
python -m gamesmanmpi_amd.build >/dev/null
mkdir -p _exp
for n in "$@"; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Igamesmanmpi_amd/csrc -DGM_EXP=$n \
    -c gamesmanmpi_amd/csrc/dense_sub.hip -o _exp/dense_sub_$n.o
  objs=$(ls gamesmanmpi_amd/_build/*.o | grep -v dense_sub.o)
  hipcc -shared -fPIC --offload-arch=gfx950 $objs _exp/dense_sub_$n.o -o _exp/libgm_exp$n.so \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo _exp/libgm_exp$n.so
done
