#!/bin/bash
# The bench line and its rocprofv3 kernel trace + stats from the same box.
export TMPDIR=/tmp
O=$(pwd)/gpurun_out
tools/gpu_steps.sh \
  "300:bench:python bench.py" \
  "300:prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-toot"
