tools/gpu_steps.sh \
  "600:pytest_new:python -u -m pytest tests/test_graph.py tests/test_cli.py -x -v --timeout 300 --timeout-method thread"
