tools/gpu_steps.sh \
  "600:pytest_sharded:python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -k dense" \
  "300:loop_b1:GM_OPT_DIST_BATCH=1 python tools/solve_timed.py subtract 8 4 8" \
  "300:loop_b4:GM_OPT_DIST_BATCH=4 python tools/solve_timed.py subtract 8 4 8" \
  "300:loop_b8:GM_OPT_DIST_BATCH=8 python tools/solve_timed.py subtract 8 4 8" \
  "300:loop2_b4:GM_OPT_DIST_BATCH=4 python tools/solve_timed.py subtract 8 4 2" \
&& tools/gpu_profile_round.sh r01
