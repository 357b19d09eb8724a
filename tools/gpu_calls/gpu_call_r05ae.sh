#!/bin/bash
# Round 5: per-tier kernel trace of the bench command with the four-wave thin-tier kernel off (0)
# and on (256 groups).
R=$(pwd)
O=$R/gpurun_out/r05ae
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "300:r05ae/kt0:GM_BOX_THIN_GROUPS=0 rocprofv3 --kernel-trace --output-format csv -d $O/kt0 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r05ae/kt256:GM_BOX_THIN_GROUPS=256 rocprofv3 --kernel-trace --output-format csv -d $O/kt256 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
)
tools/gpu_steps.sh "${steps[@]}"
