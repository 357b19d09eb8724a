#!/bin/bash
# Round 5: the four-wave thin-tier kernel with a barrier every K = 1 / 2 / 4 steps (lag S2 + K - 1):
# per-tier kernel trace with it on (tiers <= 256 groups), and its parity test per K.
R=$(pwd)
O=$R/gpurun_out/r05ag
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "300:r05ag/test_k2:GM_LIB_PATH=_exp/libgm_k2.so python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sharded.py -k four_wave"
  "300:r05ag/test_k4:GM_LIB_PATH=_exp/libgm_k4.so python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sharded.py -k four_wave"
  "300:r05ag/kt1:GM_BOX_THIN_GROUPS=256 rocprofv3 --kernel-trace --output-format csv -d $O/kt1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r05ag/kt2:GM_LIB_PATH=_exp/libgm_k2.so GM_BOX_THIN_GROUPS=256 rocprofv3 --kernel-trace --output-format csv -d $O/kt2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r05ag/kt4:GM_LIB_PATH=_exp/libgm_k4.so GM_BOX_THIN_GROUPS=256 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r05ag/kt0:GM_BOX_THIN_GROUPS=0 rocprofv3 --kernel-trace --output-format csv -d $O/kt0 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
)
tools/gpu_steps.sh "${steps[@]}"
