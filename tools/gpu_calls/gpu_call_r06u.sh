#!/bin/bash
# Round 6: the sharded sparse path inserts and looks up a rank's whole receive buffer of a tier in
# one launch (insert_bins_kernel / lookup_bins_kernel).  Parity of the sparse suites incl. the
# multi-process IPC tests, then Toot 6x4 on 8 virtual ranks with a kernel trace.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06u
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "700:r06u/parity:$P tests/test_gpu_parity.py tests/test_gpu_othello8.py tests/test_gpu_sharded.py tests/test_gpu_multiproc.py -k 'toot or othello or sparse or f2o or four or ttt'"
  "400:r06u/toot_g8:python3 -u tools/solve_timed.py toot 6 4 3 8"
  "300:r06u/othello_g8:python3 -u tools/solve_timed.py othello 4 4 5 8"
  "400:r06u/kt_g8:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_g8 -o run -- python3 tools/solve_timed.py toot 6 4 2 8"
)
tools/gpu_steps.sh "${steps[@]}"
