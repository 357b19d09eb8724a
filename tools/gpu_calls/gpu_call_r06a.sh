#!/bin/bash
# Round 6: the four-wave kernel on EVERY box-tier (GM_BOX_THIN_GROUPS above the largest tier)
# against the default two-wave kernel: kernel traces of the bench, then the full-table parity
# test with the four-wave kernel everywhere.
R=$(pwd)
O=$R/gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "300:r06a/bench0:python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r06a/kt_all4:GM_BOX_THIN_GROUPS=10000000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_all4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r06a/kt_default:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "300:r06a/test_all4:GM_BOX_THIN_GROUPS=10000000 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k subtract_8_heaps_full_table"
)
tools/gpu_steps.sh "${steps[@]}"
