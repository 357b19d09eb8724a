#!/bin/bash
# sparse engine: MLP kernels (NB children's probes in flight per lane) vs the plain ones
mkdir -p gpurun_out/r04l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for nb in 0 4 6 8 12 16; do
  GM_SPARSE_MLP=$nb timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04l/mlp$nb.log 2>&1 || exit 1
done
for nb in 0 4 8; do
  GM_SPARSE_MLP=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04l/kt$nb -o run -- python3 tools/solve_timed.py toot 6 4 3 > gpurun_out/r04l/kt$nb.log 2>&1 || exit 1
done
