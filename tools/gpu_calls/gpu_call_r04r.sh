#!/bin/bash
mkdir -p gpurun_out/r04r
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
GM_GRAPH_TRACE=1 timeout -k 10 100 python tools/graph_enum_time.py 16 16 > gpurun_out/r04r/fs_$i.log 2>&1 || exit 1
GM_GRAPH_START=spawn GM_GRAPH_TRACE=1 timeout -k 10 100 python tools/graph_enum_time.py 16 16 > gpurun_out/r04r/sp_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04r/pytest_graph.log 2>&1
