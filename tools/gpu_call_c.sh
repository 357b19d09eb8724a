tools/gpu_steps.sh \
  "600:pytest_gpu:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "300:toot_timed:python tools/solve_timed.py toot 6 4 3" \
  "300:prof_toot2:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_toot2 -o run -- python3 tools/solve_timed.py toot 6 4 2" \
  "300:oth_timed:python tools/solve_timed.py othello 4 4 3"
