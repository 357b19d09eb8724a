#!/bin/bash
# Round 6: the sharded backward reads the slots the forward inserts recorded (tables that kept their size).
# Parity of the sparse suites (incl. the multi-process IPC tests), Toot
# 6x4 and Othello 4x4 on 8 virtual ranks, Toot 6x4 and Othello 8x8 on one GPU, kernel trace.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06aj
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "700:r06aj/parity:$P tests/test_gpu_parity.py tests/test_gpu_othello8.py tests/test_gpu_sharded.py tests/test_gpu_multiproc.py -k 'toot or othello or sparse or f2o or four or ttt'"
  "400:r06aj/toot_g8:python3 -u tools/solve_timed.py toot 6 4 3 8"
  "300:r06aj/othello_g8:python3 -u tools/solve_timed.py othello 4 4 5 8"
  "300:r06aj/toot_g1:python3 -u tools/solve_timed.py toot 6 4 4"
  "300:r06aj/othello8:python3 -u tools/othello8_scale.py 16 --ranks 8 --repeats 2"
  "400:r06aj/kt_g8:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_g8 -o run -- python3 tools/solve_timed.py toot 6 4 2 8"
)
tools/gpu_steps.sh "${steps[@]}"
