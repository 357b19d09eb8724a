#!/bin/bash
# Round 6: Othello 8x8 at 12 empties vs the graph path, endgame scale on the device (seed-5
# playout roots), the default bench line (Toot positions computed vs counted, symmetry off).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
mkdir -p gpurun_out/r06e
steps=(
  "400:r06e/othello8_12:$P tests/test_gpu_othello8.py -k endgame_12"
  "400:r06e/scale_14_16:python3 -u tools/othello8_scale.py 14 15 16 --ranks 8"
  "600:r06e/scale_17_18:python3 -u tools/othello8_scale.py 17 18 --repeats 1"
  "600:r06e/bench:python3 bench.py"
)
tools/gpu_steps.sh "${steps[@]}"
