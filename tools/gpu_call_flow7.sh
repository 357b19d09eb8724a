#!/bin/bash
# one GPU call: tiered (6) vs one-launch dataflow (7) dense kernels on the 7-heap game (2^28),
# whose tiers are about one G = 8 rank's share of the 8-heap game's
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "120:h7_tiered:GM_OPT_SUB_INTERLEAVE=6 python -u tools/solve_timed.py subtract 7 6" \
  "120:h7_flow:GM_OPT_SUB_INTERLEAVE=7 python -u tools/solve_timed.py subtract 7 6" \
  "120:h6_tiered:GM_OPT_SUB_INTERLEAVE=6 python -u tools/solve_timed.py subtract 6 6" \
  "120:h6_flow:GM_OPT_SUB_INTERLEAVE=7 python -u tools/solve_timed.py subtract 6 6"
