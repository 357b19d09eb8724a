#!/bin/bash
# Round 5: Othello 8x8 endgame through the explicit-graph path (host walk, GPU resolve): the GPU
# test against the reference-plugin golden, and the launcher's root line with its time.
set -o pipefail
mkdir -p gpurun_out/r05ah
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_graph.py -k "8x8" \
    > gpurun_out/r05ah/pytest_othello8.txt 2>&1 || exit 1
( time timeout -k 10 300 python -u solver_launcher.py tests/plugins/othello8_endgame.py ) > gpurun_out/r05ah/launcher_othello8.txt 2>&1 || exit 1
