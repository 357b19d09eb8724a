#!/bin/bash
# Round 6: Othello 8x8 with the bitboard move generator (games.hpp DescOthello8::legal /
# flips_at) and classify's step counts, on the fused self-rank kernels; the bucket path
# (GM_SPARSE_SELF_FUSED=0) with the same generator for comparison.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06m
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "500:r06m/othello8_tests:$P tests/test_gpu_othello8.py tests/test_gpu_multiproc.py -k 'othello8 or 8x8'"
  "300:r06m/scale_fused:python3 -u tools/othello8_scale.py 14 16 --repeats 3"
  "300:r06m/scale_bucket:GM_SPARSE_SELF_FUSED=0 python3 -u tools/othello8_scale.py 16 --repeats 3"
  "300:r06m/kt_fused:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_fused -o run -- python3 tools/othello8_scale.py 15 --repeats 2"
)
tools/gpu_steps.sh "${steps[@]}"
