#!/bin/bash
# one GPU call: Othello 4x4 replay kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "120:oth_kt:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/oth_kt -- python3 -u tools/solve_timed.py othello 4 4 4"
