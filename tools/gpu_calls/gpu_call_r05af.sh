#!/bin/bash
# Round 5: the four-wave thin-tier kernel forced on (test), and the default paths' split tests.
set -o pipefail
mkdir -p gpurun_out/r05af
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_sharded.py -k "four_wave or graph_and_eager" \
    > gpurun_out/r05af/pytest.txt 2>&1 || exit 1
