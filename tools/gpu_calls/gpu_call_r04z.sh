#!/bin/bash
# graph walk: workers pinned one per physical core (GM_GRAPH_PIN) vs left to the scheduler
mkdir -p gpurun_out/r04z
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
GM_GRAPH_PIN=1 timeout -k 10 100 python tools/graph_enum_time.py 16 16 > gpurun_out/r04z/pin_$i.log 2>&1 || exit 1
timeout -k 10 100 python tools/graph_enum_time.py 16 16 > gpurun_out/r04z/nopin_$i.log 2>&1 || exit 1
done
