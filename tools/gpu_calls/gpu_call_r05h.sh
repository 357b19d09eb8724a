#!/bin/bash
# Round 5: per-launch kernel trace of the bench command (per-box-tier times)
# and Toot 6x4 replays with and without the kernel tracer on the same box (item 2).
TAG=r05h
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="python3 tools/solve_timed.py toot 6 4 6"
steps=(
  "200:$TAG/toot_plain:$P"
  "200:$TAG/toot_kt:rocprofv3 --kernel-trace --output-format csv -d $O/toot_kt -o run -- $P"
  "300:$TAG/bench_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_kt -o run -- python3 bench.py --no-cpu-baseline --no-toot"
  "400:$TAG/bench:python3 bench.py"
)
tools/gpu_steps.sh "${steps[@]}"
