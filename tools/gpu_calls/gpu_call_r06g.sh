#!/bin/bash
# Round 6: the 128-bit insert without acquire / release -- parity (10 / 12 empties, IPC
# processes), the 15-empty kernel trace, the 14 / 16-empty scale runs; and the Toot replay
# refill's write bytes (a PMC pass over a synced solve + a replay).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06g
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "400:r06g/othello8_tests:$P tests/test_gpu_othello8.py"
  "300:r06g/othello8_ipc:$P tests/test_gpu_multiproc.py -k othello8"
  "300:r06g/o8_trace:rocprofv3 --kernel-trace --stats --output-format csv -d $O/o8 -o run -- python3 tools/othello8_scale.py 15 --repeats 2"
  "500:r06g/scale:python3 -u tools/othello8_scale.py 14 16 --ranks 8"
  "150:r06g/refill_pmc:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/refill -o run -- python3 tools/solve_timed.py toot 6 4 2"
)
tools/gpu_steps.sh "${steps[@]}"
