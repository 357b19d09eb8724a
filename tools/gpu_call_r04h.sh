#!/bin/bash
# graph walk (peer-mesh workers, pipelined numbering) on the box's CPU share
mkdir -p gpurun_out/r04h
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
GM_GRAPH_TRACE=1 timeout -k 10 200 python tools/graph_enum_time.py 16 16 15 12 16 > gpurun_out/r04h/graph_enum.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04h/pytest_graph.log 2>&1
