#!/bin/bash
# one GPU call: sparse-engine replay (repeat solves without host round trips): parity and timing
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300:replay_tests:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'replay or othello or toot_small or four_to_one or toot_4x4'" \
  "120:replay_oth:python -u tools/solve_timed.py othello 4 4 6" \
  "120:replay_oth_off:GM_SPARSE_REPLAY=0 python -u tools/solve_timed.py othello 4 4 4" \
  "200:replay_toot:python -u tools/solve_timed.py toot 6 4 4"
