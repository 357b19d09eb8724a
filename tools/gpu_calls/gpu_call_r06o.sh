#!/bin/bash
# Round 6 (measurement only): the K128 insert's publish wait -- the shipped library against a
# variant built without the s_waitcnt before the publish (gamesmanmpi_amd/_variants/, an upper
# bound of what a protocol without that wait could gain; the variant is not correct in general).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06o
mkdir -p $O
V=$(pwd)/gamesmanmpi_amd/_variants/libgmsolve_nowait.so
steps=(
  "300:r06o/default_a:python3 -u tools/othello8_scale.py 15 16 --repeats 3"
  "300:r06o/nowait_a:GM_LIB_PATH=$V python3 -u tools/othello8_scale.py 15 16 --repeats 3"
  "300:r06o/default_b:python3 -u tools/othello8_scale.py 16 --repeats 3"
  "300:r06o/kt_nowait:GM_LIB_PATH=$V rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_nowait -o run -- python3 tools/othello8_scale.py 15 --repeats 2"
)
tools/gpu_steps.sh "${steps[@]}"
