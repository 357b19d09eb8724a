#!/bin/bash
# round-end rehearsal: the driver's default bench line, smoke(), the GPU suite
mkdir -p gpurun_out/r04k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r04k/bench.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04k/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04k/pytest_gpu.log 2>&1
