#!/bin/bash
# Round 5: full GPU suite, smoke, default bench, and the multi-process bench rehearsal.
set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05o/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05o/smoke.txt 2>&1 || exit 1
