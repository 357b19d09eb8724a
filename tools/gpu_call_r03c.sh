#!/bin/bash
# round 3: the two-half-walker option (12) -- parity on 3..6 heaps, every tier, the 2^32
# digest -- and its time against the walker (10), alternating.
tools/gpu_steps.sh \
  "300:pytest_wh:python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k 'variants or every_tier'" \
  "200:time_wh:python -u tools/quick_time.py 3,256,10,2 3,256,12,2 3,256,10,2 3,256,12,2 3,256,6,2"
