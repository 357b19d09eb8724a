#!/bin/bash
# one GPU call: the latency variant of the b4 tier kernel (all child loads up front) for tiers of
# at most GM_B4_LAT blocks: parity with every tier on it, then timing at several thresholds
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300:lat_tests:GM_B4_LAT=100000000 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'subtract' tests/test_gpu_sharded.py -k 'dense'" \
  "100:lat0:GM_B4_LAT=0 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:lat2k:GM_B4_LAT=2048 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:lat8k:GM_B4_LAT=8192 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:lat32k:GM_B4_LAT=32768 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:latall:GM_B4_LAT=100000000 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:h7_lat0:GM_B4_LAT=0 python -u tools/solve_timed.py subtract 7 4" \
  "100:h7_latall:GM_B4_LAT=100000000 python -u tools/solve_timed.py subtract 7 4" \
  "300:solo_lat0:GM_B4_LAT=0 python -u tools/solo_variants.py 8" \
  "300:solo_latall:GM_B4_LAT=100000000 python -u tools/solo_variants.py 8"
