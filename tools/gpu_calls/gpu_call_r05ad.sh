#!/bin/bash
# Round 5: the four-wave thin-tier kernel (box_tier4_kernel): parity of the full 2^32 table and
# the split engine, then N = 1 kernel ms by thin-tier threshold (GM_BOX_THIN_GROUPS; 0 = off).
set -o pipefail
mkdir -p gpurun_out/r05ad
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "subtract_8 or box" \
    > gpurun_out/r05ad/pytest_parity.txt 2>&1 || exit 1
for t in 0 256 64 128 0 256 192; do
  echo "GM_BOX_THIN_GROUPS=$t" >> gpurun_out/r05ad/thin.txt
  GM_BOX_THIN_GROUPS=$t timeout -k 10 120 python -u tools/box_variants.py gamesmanmpi_amd/libgmsolve.so >> gpurun_out/r05ad/thin.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box_split" \
    > gpurun_out/r05ad/pytest_split.txt 2>&1 || exit 1
