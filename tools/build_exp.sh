#!/bin/bash
# Development aid: build libgmsolve variants with dense_sub.hip compiled under
# -DGM_EXP=<n> into _exp/libgm_exp<n>.so (load with GM_LIB_PATH=...).  A name of
# the form <tag>=<flags> builds _exp/libgm_<tag>.so with those -D flags instead,
# e.g. "wk1=-DGM_WK_WAVES=1".
set -e
cd "$(dirname "$0")/.."
python -m gamesmanmpi_amd.build >/dev/null
mkdir -p _exp
for n in "$@"; do
  if [[ "$n" == *=* ]]; then tag="${n%%=*}"; flags="${n#*=}"; else tag="exp$n"; flags="-DGM_EXP=$n"; fi
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Igamesmanmpi_amd/csrc $flags \
    -c gamesmanmpi_amd/csrc/dense_sub.hip -o _exp/dense_sub_$tag.o
  objs=$(ls gamesmanmpi_amd/_build/*.o | grep -v dense_sub.o)
  hipcc -shared -fPIC --offload-arch=gfx950 $objs _exp/dense_sub_$tag.o -o _exp/libgm_$tag.so \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo _exp/libgm_$tag.so
done
