#!/bin/bash
# Sharded dense solve: GPU parity (both block owners), per-rank solo timing of both
# owners, and the bench's sharded path with 8 loopback ranks under each owner.
tools/gpu_steps.sh \
 "600:pytest_owner:python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -k 'tier_balanced or dense'" \
 "300:owner_solo:python -u tools/owner_solo.py 8" \
 "200:bench_v8_o0:python bench.py --virtual-ranks 8 --no-cpu-baseline --no-toot --dist-owner 0" \
 "200:bench_v8_o1:python bench.py --virtual-ranks 8 --no-cpu-baseline --no-toot --dist-owner 1"
