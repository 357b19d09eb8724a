#!/bin/bash
# round 3, one GPU call: the Othello-symmetry / launcher / graph tests, the sort+unique
# dedup measurement (tools/sort_dedup.hip), and fresh PMC passes + a kernel trace of the
# mirror-reduced Toot-and-Otto 6x4 sparse solve (one solve per pass).
O=$(pwd)/gpurun_out
export TMPDIR=/tmp
T="python3 tools/solve_timed.py toot 6 4 1"
tools/gpu_steps.sh \
  "600:pytest_oth:python -u -m pytest tests/test_gpu_parity.py tests/test_graph.py tests/test_gpu_sharded.py tests/test_cli.py -m gpu -v --timeout 300 --timeout-method thread -k 'othello or graph or sparse or launcher'" \
  "120:sortdedup:tools/_bin/sort_dedup" \
  "150:toot_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/toot_kt -o run -- python3 tools/solve_timed.py toot 6 4 3" \
  "150:toot_fetch:timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/toot_fetch -o run -- $T" \
  "150:toot_write:timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/toot_write -o run -- $T" \
  "150:toot_hit:timeout -s KILL 140 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/toot_hit -o run -- $T" \
  "150:toot_atomic:timeout -s KILL 140 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --output-format csv -d $O/toot_atomic -o run -- $T"
