#!/bin/bash
# Round 6 experiment: Othello 8x8 at 16 empties, the 128-bit lookup with the score load issued
# beside the key load (new) against after the compare (old, _exp/libgm_old.so), alternated.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06au
out=gpurun_out/r06au/spec_score.txt
for i in 1 2; do
  echo "== old" >> $out
  GM_LIB_PATH=_exp/libgm_old.so timeout -k 10 120 python3 tools/othello8_scale.py 16 --repeats 3 >> $out 2>&1 || exit 1
  echo "== new" >> $out
  timeout -k 10 120 python3 tools/othello8_scale.py 16 --repeats 3 >> $out 2>&1 || exit 1
done
