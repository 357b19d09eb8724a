#!/bin/bash
# Round 6: per-workgroup counter atomics (block_add) and capped grids (grid_counted) in the sparse
# kernels that end by adding to one counter; the bucket kernels' count pass flushes its LDS
# histogram once per workgroup.  Parity of the sparse suites, then Toot 6x4 on one GPU and on
# 8 virtual ranks, Othello 8x8, and a kernel trace of the sharded Toot solve.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06t
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "600:r06t/parity:$P tests/test_gpu_parity.py tests/test_gpu_othello8.py tests/test_gpu_sharded.py -k 'toot or othello or sparse or f2o or four or ttt'"
  "300:r06t/toot_g1:python3 -u tools/solve_timed.py toot 6 4 4"
  "400:r06t/toot_g8:python3 -u tools/solve_timed.py toot 6 4 3 8"
  "300:r06t/othello8:python3 -u tools/othello8_scale.py 15 16 --repeats 3"
  "400:r06t/kt_g8:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_g8 -o run -- python3 tools/solve_timed.py toot 6 4 2 8"
  "300:r06t/kt_g1:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_g1 -o run -- python3 tools/solve_timed.py toot 6 4 4"
)
tools/gpu_steps.sh "${steps[@]}"
