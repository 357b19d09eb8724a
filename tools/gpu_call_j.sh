tools/gpu_steps.sh \
  "600:pytest_sharded:python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -k sparse" \
  "300:toot_g8:python tools/solve_timed.py toot 6 4 2 8" \
  "300:toot_g2:python tools/solve_timed.py toot 6 4 2 2" \
  "300:oth_g8:python tools/solve_timed.py othello 4 4 2 8"
