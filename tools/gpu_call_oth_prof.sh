#!/bin/bash
# one GPU call: sparse parity subset, then Othello 4x4 replay timing and kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:sp_tests:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'replay or othello or toot_small or toot_4x4 or four_to_one or symmetry'" \
  "120:oth_time:python -u tools/solve_timed.py othello 4 4 6" \
  "120:oth_kt:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/oth_kt -- python3 -u tools/solve_timed.py othello 4 4 4"
