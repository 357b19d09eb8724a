#!/bin/bash
# one GPU call: sparse parity + timing, then the bench line (GPU_MAX_HW_QUEUES 8 from bench.py)
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300:sparse_tests:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'replay or othello or toot or four_to_one or ttt'" \
  "120:time_oth:python -u tools/solve_timed.py othello 4 4 6" \
  "400:bench:python bench.py"
