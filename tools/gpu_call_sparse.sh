#!/bin/bash
# one GPU call: sparse engines -- replay (repeat solves without host round trips) and the
# Toot mirror-symmetry reduction: parity tests, then timing
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "400:sparse_tests:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k 'replay or othello or toot or four_to_one or ttt'" \
  "300:sparse_sharded:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -k 'sparse'" \
  "120:time_oth:python -u tools/solve_timed.py othello 4 4 6" \
  "200:time_toot:python -u tools/solve_timed.py toot 6 4 4" \
  "200:time_toot_nosym:GM_OPT_SYMMETRY=0 python -u tools/solve_timed.py toot 6 4 3"
