#!/bin/bash
# Round 6: the hash-sharded sparse path's cost for Toot 6x4 (config 3) -- 8 virtual ranks on one
# GPU (every rank's kernels back to back, loopback copies) against the one-GPU engine, with a
# kernel trace of the sharded solves.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06q
mkdir -p $O
steps=(
  "300:r06q/toot_g1:python3 -u tools/solve_timed.py toot 6 4 3"
  "400:r06q/toot_g8:python3 -u tools/solve_timed.py toot 6 4 3 8"
  "400:r06q/kt_g8:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_g8 -o run -- python3 tools/solve_timed.py toot 6 4 2 8"
)
tools/gpu_steps.sh "${steps[@]}"
