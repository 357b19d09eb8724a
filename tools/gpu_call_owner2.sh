#!/bin/bash
# one GPU call: Othello custom-root parity, then per-rank solo times under both block owners
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "200:oth_roots:python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k 'othello_custom'" \
  "500:owner_solo:python -u tools/owner_solo.py 8"
