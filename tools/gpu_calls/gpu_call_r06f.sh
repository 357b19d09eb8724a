#!/bin/bash
# Round 6: where the Othello 8x8 forward pass spends its time (kernel trace of the 15-empty
# solve), and the Toot replay refill's write bytes (PMC pass over a synced solve + a replay).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06f
mkdir -p $O
steps=(
  "300:r06f/o8_trace:GM_TRACE=1 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o8 -o run -- python3 tools/othello8_scale.py 15 --repeats 2"
  "150:r06f/refill_pmc:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/refill -o run -- python3 tools/solve_timed.py toot 6 4 2"
)
tools/gpu_steps.sh "${steps[@]}"
