tools/gpu_steps.sh \
  "150:toot_trace:GM_TRACE=1 python -u tools/solve_timed.py toot 6 4 3" \
  "600:pytest_gpu:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
