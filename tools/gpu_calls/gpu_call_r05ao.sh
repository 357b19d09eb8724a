#!/bin/bash
# Round 5: Othello 8x8 endgames of 12 and 13 empty squares through the graph path (launcher
# root line and wall time; the walk stops itself if its projection passes the limits).
set -o pipefail
mkdir -p gpurun_out/r05ao
for r in 30380028503841784646bfd6afc6be000200 30381c2c503841784646a1d2afc6be000100; do
  echo "root $r" >> gpurun_out/r05ao/othello8.txt
  ( time GM_OTHELLO8_ROOT=$r GM_GRAPH_TRACE=1 timeout -k 10 400 python -u solver_launcher.py tests/plugins/othello8_endgame.py ) \
      >> gpurun_out/r05ao/othello8.txt 2>&1 || exit 1
done
