#!/bin/bash
# graph walk with overlapping levels: chunk / nice scan on the box's CPU share
mkdir -p gpurun_out/r04i
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 100 python tools/graph_enum_time.py 16 > gpurun_out/r04i/warm.log 2>&1 || exit 1
for c in 256 64 32; do for n in 0 2; do
  GM_GRAPH_CHUNK=$c GM_GRAPH_NICE=$n GM_GRAPH_TRACE=1 timeout -k 10 100 python tools/graph_enum_time.py 16 16 16 > gpurun_out/r04i/graph_c${c}_n$n.log 2>&1 || exit 1
done; done
