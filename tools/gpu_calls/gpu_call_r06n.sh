#!/bin/bash
# Round 6: does the 17-empty root of the seed-5 playout fit one GPU now that the one-rank
# solve keeps no key lists (round 6's first try ran out of memory)?
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06n
steps=(
  "400:r06n/scale17:GM_TRACE=1 python3 -u tools/othello8_scale.py 17 --repeats 2"
)
tools/gpu_steps.sh "${steps[@]}"
