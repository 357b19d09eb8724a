#!/bin/bash
mkdir -p gpurun_out/r04q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 32 16; do
GM_SPARSE_CROWS=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q/kt$r -o run -- python3 tools/solve_timed.py toot 6 4 3 > gpurun_out/r04q/t$r.log 2>&1 || exit 1
done
