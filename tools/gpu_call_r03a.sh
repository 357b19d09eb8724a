tools/gpu_steps.sh \
  "900:pytest_gpu:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py"
