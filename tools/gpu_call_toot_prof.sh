#!/bin/bash
# one GPU call: Toot-and-Otto 6x4 kernel trace + stats (symmetry on, the default), and the
# same with GM_OPT_SYMMETRY=0, three solves each (the first synced, then replays)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "200:toot_sym_kt:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/toot_sym -o run -- python3 -u tools/solve_timed.py toot 6 4 3" \
  "200:toot_nosym_kt:GM_OPT_SYMMETRY=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/toot_nosym -o run -- python3 -u tools/solve_timed.py toot 6 4 3"
