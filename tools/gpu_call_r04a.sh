#!/bin/bash
# round 4: first run of the sharded box engine (virtual ranks), smoke, headline bench
set -o pipefail
mkdir -p gpurun_out/r04a
export PYTHONUNBUFFERED=1
GM_GRAPH_TRACE=1 timeout -k 10 300 python tools/graph_enum_time.py 16 16 1 > gpurun_out/r04a/graph_enum.log 2>&1
timeout -k 10 300 python tools/box_shard_time.py --reps 10 > gpurun_out/r04a/shard_time.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -k "box" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/pytest_box.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --no-toot --no-cpu-baseline > gpurun_out/r04a/bench.log 2>&1
