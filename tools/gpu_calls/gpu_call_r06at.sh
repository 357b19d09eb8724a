#!/bin/bash
# Round 6 closing profile of the headline: the default bench line on the round's last code, its
# kernel trace (rocprofv3 --kernel-trace --stats) and one --pmc pass each for FETCH_SIZE and
# WRITE_SIZE (tools/pmc_summary.py turns them into profiles/r06/r06at_subtract8_summary.json).
TAG=r06at
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "400:$TAG/bench:python3 bench.py"
  "300:$TAG/prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "120:$TAG/prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
  "120:$TAG/prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
)
tools/gpu_steps.sh "${steps[@]}"
