#!/bin/bash
# graph walk: 16 vs 15 workers (the parent numbering beside them), fork server
mkdir -p gpurun_out/r04z
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 100 python tools/graph_enum_time.py 16 15 16 15 > gpurun_out/r04z/w_$i.log 2>&1 || exit 1
done
