#!/bin/bash
# sparse engine on Toot 6x4: round-3 kernels (0), sorted lists + plain kernels (2), batch kernels (1)
mkdir -p gpurun_out/r04e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for m in 0 2 1; do
  GM_SPARSE_BATCH=$m timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04e/toot64_m$m.log 2>&1 || exit 1
done
for m in 0 2 1; do
  GM_SPARSE_BATCH=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e/kt_m$m -o run -- python3 tools/solve_timed.py toot 6 4 3 > gpurun_out/r04e/kt_m$m.log 2>&1 || exit 1
done
