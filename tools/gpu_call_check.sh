#!/bin/bash
# One GPU call after a kernel change: the full GPU parity suite, the bench line, the
# sharded loopback timing at 8 ranks and one rank's tier launches alone (G = 8).
tools/gpu_steps.sh \
 "900:pytest_gpu:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "300:bench:python bench.py" \
 "120:v8:python tools/solve_timed.py subtract 8 6 8" \
 "120:solo8_r0:GM_OPT_DIST_SOLO=1 python tools/solve_timed.py subtract 8 6 8"
