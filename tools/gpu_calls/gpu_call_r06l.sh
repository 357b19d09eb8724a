#!/bin/bash
# Round 6: Othello 8x8 on one GPU through the fused self-rank kernels (self_expand_kernel /
# self_retro_kernel, dist_sparse.hip) against the bucket path (GM_SPARSE_SELF_FUSED=0).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06l
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "500:r06l/othello8_tests:$P tests/test_gpu_othello8.py"
  "300:r06l/scale_fused:python3 -u tools/othello8_scale.py 14 16 --repeats 3"
  "300:r06l/scale_bucket:GM_SPARSE_SELF_FUSED=0 python3 -u tools/othello8_scale.py 16 --repeats 3"
  "300:r06l/kt_fused:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_fused -o run -- python3 tools/othello8_scale.py 15 --repeats 2"
)
tools/gpu_steps.sh "${steps[@]}"
